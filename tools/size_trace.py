"""Kernel timelines of C4-shaped batches at chosen sizes (one GPU).

Run under rocprofv3 --kernel-trace; every size gets 1 + reps on-device
bgv_verify calls of the first `size` sets' whole blocks of the segment, with a
short idle gap between sizes.  The call order is written to
gpurun_out/size_trace_calls.json so `--analyze TRACE.csv` can cut the trace
into calls (each call launches k_gen_scalars once) and print the timeline of
the last call of every size.

    rocprofv3 --kernel-trace -d OUT -o run --output-format csv -- python3 tools/size_trace.py --sizes 3136,12544
    python3 tools/size_trace.py --analyze OUT/.../run_kernel_trace.csv
"""
import argparse
import csv
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CALLS = os.path.join(ROOT, "gpurun_out", "size_trace_calls.json")


def run(sizes, reps, cfg, single=0):
    import numpy as np
    import torch

    import bench
    from lodestar_amd import native
    from lodestar_amd.dist import select_jobs

    dev = torch.device("cuda", 0)
    seg = bench.build_segment(list(range(max(sizes) // bench.SETS_PER_BLOCK)))
    d = native.Device(0, **cfg)
    d.gen_keys(0, bench.N_VALIDATORS, bench.SEED)
    calls = []
    for n in sizes:
        a = select_jobs(seg, list(range(n // bench.SETS_PER_BLOCK)))
        da = bench.to_device(a, torch, dev)
        sigs = torch.zeros((a["n_sets"], 192), dtype=torch.uint8, device=dev)
        d.gen_sign(da, sigs, on_device=True)
        da.update(sigs=sigs, sig_len=torch.full((a["n_sets"],), 96, dtype=torch.int32, device=dev), scalars=None)
        t = []
        for r in range(1 + reps):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            jr, _ = d.verify(da, on_device=True, want_set_codes=False)
            t.append(time.perf_counter() - t1)
            assert (jr == 1).all(), n
            calls.append(n)
        print(json.dumps({"sets": n, "ms_p50": round(float(np.median(t[1:])) * 1e3, 3)}), flush=True)
        time.sleep(0.05)
    if single:  # one host-resident set per call (bench.py single_set_latency_ms)
        arr = bench.signed(d, bench.singles(1, bench.SEED + 3500))
        t = []
        for r in range(1 + single):
            t1 = time.perf_counter()
            jr, _ = d.verify(arr, on_device=False, want_set_codes=False)
            t.append(time.perf_counter() - t1)
            assert (jr == 1).all()
            calls.append(1)
        print(json.dumps({"sets": 1, "host": True, "ms_p50": round(float(np.median(t[1:])) * 1e3, 3)}), flush=True)
    d.close()
    os.makedirs(os.path.dirname(CALLS), exist_ok=True)
    json.dump(calls, open(CALLS, "w"))


def analyze(path, calls_path):
    """the timeline of the last call of every size: the dispatches after the
    previous call's batch final exponentiation up to this call's (one
    k_batch_final per verify call; the signing calls have none)"""
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    calls = json.load(open(calls_path))
    bf = [r for r in rows if "k_batch_final" in r["Kernel_Name"]][-len(calls):]
    for ci, n in enumerate(calls):
        if ci == 0 or (ci + 1 < len(calls) and calls[ci + 1] == n):
            continue  # only the last call of each size
        t_prev, t_end = int(bf[ci - 1]["End_Timestamp"]), int(bf[ci]["End_Timestamp"])
        sel = [r for r in rows if t_prev < int(r["Start_Timestamp"]) and int(r["End_Timestamp"]) <= t_end]
        t0 = int(sel[0]["Start_Timestamp"])
        print(f"== {n} sets: device span {(t_end - t0) / 1e6:.3f} ms (first dispatch to the final exponentiation's end)")
        for r in sel:
            s_, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            print(f"  {(s_ - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s_) / 1e6:8.3f} q{r['Queue_Id']} "
                  f"{r['Kernel_Name'][:40]:40s} grid={r['Grid_Size_X']} vgpr={r.get('VGPR_Count', '')}/"
                  f"{r.get('Accum_VGPR_Count', '')} lds={r.get('LDS_Block_Size', '')} scr={r.get('Scratch_Size', '')}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="3136,12544")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cfg", default="{}", help="bgv_cfg overrides as JSON, e.g. '{\"miller\": 2}'")
    ap.add_argument("--single", type=int, default=0, help="also time this many host-resident one-set calls")
    ap.add_argument("--analyze")
    ap.add_argument("--calls", default=CALLS)
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze, a.calls)
    else:
        run([int(x) for x in a.sizes.split(",") if x], a.reps, json.loads(a.cfg), a.single)


if __name__ == "__main__":
    main()
