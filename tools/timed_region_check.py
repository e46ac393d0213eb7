"""Agreement of the bench's in-process HIP-event stage times with rocprofv3.

    python3 tools/timed_region_check.py TRACE_kernel_trace.csv BENCH.json [--inflight 3 --steps 20 --warmup 1]

The trace is `rocprofv3 --kernel-trace` of `bench.py --no-c2 --no-cpu --steps K`
(one C4 batch per step, D in flight).  Per kernel the dispatches come in bench
order: D context-priming batches, W warm-up batches, the K timed batches, then
the one_in_flight leg (1 + 5 lone batches).  For each stage's main kernel the
mean rocprof duration of the K timed dispatches is printed beside the bench's
stage time of the timed region, and the mean of the last 5 beside the bench's
isolated (one batch in flight) stage time."""
import argparse
import csv
import json
from collections import defaultdict

KERNELS = [("k_miller", "miller_loop"), ("k_hash", "hash_to_g2"), ("k_pk_chunk", "pk_gather"),
           ("k_sig", "sig_decode_subgroup"), ("k_lines", None), ("k_msm_bucket", "sig_scale")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--inflight", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    j = json.loads(open(args.bench).read().strip().splitlines()[-1])
    roof = j["roofline"]
    per_stage, iso = roof["per_stage"], roof["isolated"]["stage_ms"]
    d = defaultdict(list)
    for r in csv.DictReader(open(args.trace)):
        name = r["Kernel_Name"].split("(")[0].replace("bgv::", "").strip()
        d[name].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    first = args.inflight + args.warmup
    print(f"rocprofv3 --kernel-trace of `bench.py --no-c2 --no-cpu --steps {args.steps}` ({args.inflight} batches in flight);")
    print(f"dispatch order per kernel: {args.inflight} context-priming + {args.warmup} warm-up batches, the {args.steps} timed "
          "batches, then one_in_flight (1 + 5).")
    for k, stage in KERNELS:
        v = sorted(d.get(k, []))
        if len(v) < first + args.steps:
            continue
        timed = [(e - s) / 1e6 for s, e in v[first:first + args.steps]]
        lone = [(e - s) / 1e6 for s, e in v[-5:]]
        tm, lm = sum(timed) / len(timed), sum(lone) / len(lone)
        line = f"  {k:12s} dispatches {len(v):3d}  timed mean {tm:7.3f} ms"
        if stage:
            line += f"  bench stage {stage} {per_stage[stage]['ms']:7.3f} ms"
        line += f"  | one_in_flight mean {lm:7.3f} ms"
        if stage:
            line += f"  bench isolated {iso[stage]:7.3f} ms"
        print(line)
    print(f"bench line: {j['value']} sets/s, {j['ms_per_step']} ms per batch; dominant stage {roof['kernel']} "
          f"({roof['kernel_name']}) frac {roof['frac']}, isolated frac {roof['isolated']['frac']}; "
          f"step {roof['step_fpmul_G_per_s']} G Fp-mul/s")


if __name__ == "__main__":
    main()
