"""A/B sweep of the pipeline knobs over batch sizes (one GPU): for each
(size, bgv_cfg override set) the median on-device bgv_verify time of a
C4-shaped batch (the first `size` sets' whole blocks of the segment).  Prints
one JSON line per point.  Every override set opens its own context
(bgv_open_cfg).

    python tools/sweep_modes.py [--sizes 12544,25088,50176,100352] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MODES = {  # bgv_cfg overrides (include/bgv.h)
    "default": {},
    "bulk_cu8": {"cu_split": -8},  # the Node pool's bulk context beside a priority context (r05)
    "prio_cu8": {"cu_split": 8},  # the priority context itself on 8 reserved CUs
    "prefold1": {"prefold": 1},
    "msm4": {"msm": 4},
    "d100": {"defer_pct": 100},
    "d90": {"defer_pct": 90},
    "d60": {"defer_pct": 60},
    "msm4d100": {"msm": 4, "defer_pct": 100},
    "prefold0": {"prefold": 0},
    "bulk_cu32": {"cu_split": -32},
    "prio_cu32": {"cu_split": 32},
    "bulk_cu16": {"cu_split": -16},
    "prio_cu16": {"cu_split": 16},
    "split0": {"split": 0},
    "split0_serial": {"split": 0, "miller": 1},
    "split0_serial_msm": {"split": 0, "miller": 1, "msm": 1},
    "bulk_c4": {"split": 0, "miller": 1, "msm": 1, "pairs": 2},
    "split1_serial_msm": {"split": 1, "miller": 1, "msm": 1},
    "coop_msm": {"msm": 1},
    "split1_serial": {"split": 1, "miller": 1, "msm": 0},
    "split1_coop_msm": {"split": 1, "miller": 36, "msm": 1},
    "m2": {"miller": 2},
    "c3": {"clear_lanes": 3},
    "c9": {"clear_lanes": 9},
    "c1": {"clear_lanes": 1},
    "m4c1": {"miller": 4, "clear_lanes": 1},
    "m2c1": {"miller": 2, "clear_lanes": 1},
    "m2c3": {"miller": 2, "clear_lanes": 3},
    "m2c9": {"miller": 2, "clear_lanes": 9},
    "msm0c3": {"msm": 0, "clear_lanes": 3},
    "m4": {"miller": 4},
    "m4msm3c3": {"miller": 4, "msm": 3, "clear_lanes": 3},
    "m2msm3c3": {"miller": 2, "msm": 3, "clear_lanes": 3},
    "m4msm3c9": {"miller": 4, "msm": 3, "clear_lanes": 9},
    "m6msm3c9": {"miller": 6, "msm": 3, "clear_lanes": 9},
    "m18msm3c9": {"miller": 18, "msm": 3, "clear_lanes": 9},
    "m4msm0c3": {"miller": 4, "msm": 0, "clear_lanes": 3},
    "m4msm2c3": {"miller": 4, "msm": 2, "clear_lanes": 3},
    "m4msm4c3": {"miller": 4, "msm": 4, "clear_lanes": 3},
    "m2msm4c3": {"miller": 2, "msm": 4, "clear_lanes": 3},
    "m4msm1c9": {"miller": 4, "msm": 1, "clear_lanes": 9},
    "m4msm0c9": {"miller": 4, "msm": 0, "clear_lanes": 9},
    "msm0c9": {"msm": 0, "clear_lanes": 9},
    "msm0m2c3": {"msm": 0, "miller": 2, "clear_lanes": 3},
    "msm0m2c9": {"msm": 0, "miller": 2, "clear_lanes": 9},
    "msm2c3": {"msm": 2, "clear_lanes": 3},
    "msm2m2c3": {"msm": 2, "miller": 2, "clear_lanes": 3},
    "m6": {"miller": 6},
    "m18": {"miller": 18},
    "m36": {"miller": 36},
    "serial": {"miller": 1},
    "m6_s0": {"miller": 6, "split": 0},
    "j18": {"job_lanes": 18},
    "j6": {"job_lanes": 6},
    "timed": {"timing": 1},
    "msm0": {"msm": 0},
    "msm1": {"msm": 1},
    "msm2": {"msm": 2},
    "nodefer": {"defer_pct": 0},
    "d75": {"defer_pct": 75},
    "d25": {"defer_pct": 25},
    "s1m2c1m4": {"split": 1, "miller": 2, "clear_lanes": 1, "msm": 4},
    "s1m1c1m4": {"split": 1, "miller": 1, "clear_lanes": 1, "msm": 4},
    "s1m1c1m2": {"split": 1, "miller": 1, "clear_lanes": 1, "msm": 2},
    "s0m2": {"split": 0, "miller": 2},
    "s0m4msm": {"split": 0, "msm": 4},
    "d0": {"defer_pct": 0},
    "d50": {"defer_pct": 50},
    "d100": {"defer_pct": 100},
    "nolines": {"lines": 0},
    "p2": {"pairs": 2},
    "p2l": {"pairs": 2, "lines": 1},
    "kv3": {"miller_kv": 3},
    "kv6": {"miller_kv": 6},
    "kv9": {"miller_kv": 9},
    "kv2": {"miller_kv": 2},
    "kv0": {"miller_kv": 0},
}


def main():
    import torch

    import bench
    from lodestar_amd import native

    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="12544,25088,50176,100352")
    ap.add_argument("--modes", default=",".join(MODES))
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    seg = bench.build_segment(list(range(1024)))
    sizes = [int(x) for x in args.sizes.split(",")]
    signer = native.Device(0)
    signer.gen_keys(0, bench.N_VALIDATORS, bench.SEED)
    batches = {}
    from lodestar_amd.dist import select_jobs
    for n in sizes:
        a = select_jobs(seg, list(range(n // bench.SETS_PER_BLOCK)))
        da = bench.to_device(a, torch, dev)
        sigs = torch.zeros((a["n_sets"], 192), dtype=torch.uint8, device=dev)
        signer.gen_sign(da, sigs, on_device=True)
        da.update(sigs=sigs, sig_len=torch.full((a["n_sets"],), 96, dtype=torch.int32, device=dev), scalars=None)
        batches[n] = da
    signer.close()
    for name in args.modes.split(","):
        d = native.Device(0, **MODES[name])
        d.gen_keys(0, bench.N_VALIDATORS, bench.SEED)
        for n in sizes:
            da = batches[n]
            jr, _ = d.verify(da, on_device=True, want_set_codes=False)
            assert (jr == 1).all(), (name, n)
            t = []
            for _ in range(args.reps):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                d.verify(da, on_device=True, want_set_codes=False)
                t.append(time.perf_counter() - t1)
            ms = float(np.median(t)) * 1e3
            row = {"mode": name, "sets": n, "ms": round(ms, 3), "sets_per_s": round(n / ms * 1e3, 1)}
            row["layout"] = d.last_stats.layout()
            if MODES[name].get("timing") == 1 or n >= 65536:  # per-stage event times of the last call
                row["stage_ms"] = {k: round(v, 3) for k, v in d.last_stats.as_dict(d)["stage_ms"].items() if v > 0}
            print(json.dumps(row), flush=True)
        d.close()


if __name__ == "__main__":
    main()
