"""P processes on GPU 0 at once, each verifying its own work-balanced shard
of a C4 segment `reps` times (bgv_verify and bgv_partial + its own
combine_final), no collectives: checks that the library's results do not
depend on other processes' kernels sharing the GPU.  Prints JSON lines."""
import json
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, world, reps, timing, q):
    try:
        import torch

        import bench
        from lodestar_amd import native
        from lodestar_amd.dist import batch_job_work, select_jobs, shard_jobs
        dev = torch.device("cuda", 0)
        seg = bench.build_segment(list(range(1024)), seed=bench.SEED)
        shards = shard_jobs(batch_job_work(seg), world)
        d = native.Device(0, timing=timing)
        d.gen_keys(0, bench.N_VALIDATORS, bench.SEED)
        a = select_jobs(seg, shards[rank])
        da = bench.to_device(a, torch, dev)
        sigs = torch.zeros((a["n_sets"], 192), dtype=torch.uint8, device=dev)
        d.gen_sign(da, sigs, on_device=True)
        da.update(sigs=sigs, sig_len=torch.full((a["n_sets"],), 96, dtype=torch.int32, device=dev), scalars=None)
        res = []
        for _ in range(reps):
            jr, sc = d.verify(da, on_device=True, want_set_codes=True)
            part, _, jobs, pok = d.partial(da, on_device=True)
            comb = d.combine_final([part])
            res.append([bool((jr == 1).all()), int((jr != 1).sum()), sorted(set(int(c) for c in sc if c))[:4], bool(comb)])
        q.put((rank, {"sets": a["n_sets"], "layout": d.last_stats.layout(), "runs": res}))
        d.close()
    except BaseException as e:
        q.put((rank, repr(e)))


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    timing = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, world, reps, timing, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r in sorted(out):
        print(json.dumps({"world": world, "timing": timing, "rank": r, "result": out[r]}), flush=True)


if __name__ == "__main__":
    main()
