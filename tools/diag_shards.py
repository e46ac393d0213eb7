"""One process, one context: a C4 segment split into `world` work-balanced
shards (dist.shard_jobs), each shard through bgv_partial, then
bgv_combine_final over all partials -- the N>1 bench path without the
collectives.  Also each shard alone through bgv_verify.  Prints JSON lines."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from lodestar_amd import native
    from lodestar_amd.dist import batch_job_work, select_jobs, shard_jobs
    blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    worlds = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "2,4,8").split(",")]
    dev = torch.device("cuda", 0)
    seg = bench.build_segment(list(range(blocks)), seed=bench.SEED)
    for timing in (0, 1):
        d = native.Device(0, timing=timing)
        d.gen_keys(0, bench.N_VALIDATORS, bench.SEED)
        for world in worlds:
            shards = shard_jobs(batch_job_work(seg), world)
            parts, ok_each = [], []
            for r in range(world):
                a = select_jobs(seg, shards[r])
                da = bench.to_device(a, torch, dev)
                sigs = torch.zeros((a["n_sets"], 192), dtype=torch.uint8, device=dev)
                d.gen_sign(da, sigs, on_device=True)
                da.update(sigs=sigs, sig_len=torch.full((a["n_sets"],), 96, dtype=torch.int32, device=dev), scalars=None)
                jr, _ = d.verify(da, on_device=True, want_set_codes=False)
                ok_each.append(bool((jr == 1).all()))
                part, _, jobs, pok = d.partial(da, on_device=True)
                parts.append(part)
            comb = d.combine_final(parts)
            print(json.dumps({"timing": timing, "world": world, "sets_per_shard": a["n_sets"], "verify_each": ok_each,
                              "combined": bool(comb), "layout": d.last_stats.layout()}), flush=True)
        d.close()


if __name__ == "__main__":
    main()
