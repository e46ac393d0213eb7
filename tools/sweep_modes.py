"""A/B sweep of the pipeline knobs over batch sizes (one GPU): for each
(size, knob set) the median on-device bgv_verify time of a C4-shaped batch
(the first `size` sets' whole blocks of the segment).  Prints one JSON line
per point.  Knobs are read by bgv_open, so every point opens its own context.

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

MODES = {
    "default": {},
    "split0": {"BGV_SPLIT": "0"},
    "split0_serial": {"BGV_SPLIT": "0", "BGV_MILLER": "serial"},
    "split0_serial_msm": {"BGV_SPLIT": "0", "BGV_MILLER": "serial", "BGV_MSM": "1"},
    "bulk_c4": {"BGV_SPLIT": "0", "BGV_MILLER": "serial", "BGV_MSM": "1", "BGV_PAIRS": "2"},
    "split1_serial_msm": {"BGV_SPLIT": "1", "BGV_MILLER": "serial", "BGV_MSM": "1"},
    "coop_msm": {"BGV_MSM": "1"},
    "split1_serial": {"BGV_SPLIT": "1", "BGV_MILLER": "serial", "BGV_MSM": "0"},
    "split1_coop_msm": {"BGV_SPLIT": "1", "BGV_MILLER": "coop", "BGV_MSM": "1"},
    "m6": {"BGV_MILLER": "6"},
    "m18": {"BGV_MILLER": "18"},
    "m36": {"BGV_MILLER": "36"},
    "serial": {"BGV_MILLER": "serial"},
    "m6_s0": {"BGV_MILLER": "6", "BGV_SPLIT": "0"},
    "j18": {"BGV_JOB_LANES": "18"},
    "j6": {"BGV_JOB_LANES": "6"},
    "isolated": {"BGV_OVERLAP": "0", "BGV_TIMING": "1"},
    "d1": {"BGV_DEFER": "1"},
    "d2": {"BGV_DEFER": "2"},
    "d4": {"BGV_DEFER": "4"},
    "d5": {"BGV_DEFER": "5"},
    "d6": {"BGV_DEFER": "6"},
    "noprio": {"BGV_PRIO": "0"},
}
KNOBS = ("BGV_SPLIT", "BGV_MILLER", "BGV_MSM", "BGV_PAIRS", "BGV_PREFOLD", "BGV_JOB_LANES", "BGV_OVERLAP", "BGV_TIMING",
         "BGV_DEFER", "BGV_PRIO")


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
        for k in KNOBS:
            os.environ.pop(k, None)
        os.environ.update(MODES[name])
        d = native.Device(0)
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
            if os.environ.get("BGV_TIMING") == "1" or n >= 65536:  # per-stage event times of the last call
                row["stage_ms"] = {k: round(v, 3) for k, v in d.last_stats.as_dict(d)["stage_ms"].items() if v > 0}
            print(json.dumps(row), flush=True)
        d.close()


if __name__ == "__main__":
    main()
