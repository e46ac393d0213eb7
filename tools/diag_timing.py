"""Verify C4-shaped batches of whole blocks at chosen sizes with the stage-timing
events off and on (bgv_cfg.timing), on device; prints one JSON line each."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from lodestar_amd import native
    from lodestar_amd.dist import select_jobs
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "3136,12544,25088").split(",")]
    dev = torch.device("cuda", 0)
    seg = bench.build_segment(list(range(max(sizes) // bench.SETS_PER_BLOCK)))
    for timing in (0, 1):
        d = native.Device(0, timing=timing)
        d.gen_keys(0, bench.N_VALIDATORS, bench.SEED)
        for n in sizes:
            a = select_jobs(seg, list(range(n // bench.SETS_PER_BLOCK)))
            da = bench.to_device(a, torch, dev)
            sigs = torch.zeros((a["n_sets"], 192), dtype=torch.uint8, device=dev)
            d.gen_sign(da, sigs, on_device=True)
            da.update(sigs=sigs, sig_len=torch.full((a["n_sets"],), 96, dtype=torch.int32, device=dev), scalars=None)
            jr, sc = d.verify(da, on_device=True, want_set_codes=True)
            bad = [int(j) for j in range(len(jr)) if jr[j] != 1][:5]
            print(json.dumps({"timing": timing, "sets": n, "all_valid": bool((jr == 1).all()), "first_bad_jobs": bad,
                              "bad_codes": sorted(set(int(c) for c in sc if c != 0))[:5],
                              "layout": d.last_stats.layout()}), flush=True)
        d.close()


if __name__ == "__main__":
    main()
