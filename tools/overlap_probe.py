"""Probe: do two C4 batches in flight on ONE GPU (two contexts, one host
thread each) finish sooner than the same batches back to back?  The second
batch's phase 1 (hash, pubkeys, decode) can use the SIMDs the first batch's
one-wave Miller phase leaves idle.  Prints one JSON line per configuration.
Run on the GPU box: python tools/overlap_probe.py [--ctx 2] [--steps 8]"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=2)
    ap.add_argument("--steps", type=int, default=8, help="batches per context")
    ap.add_argument("--blocks", type=int, default=1024)
    ap.add_argument("--cfg", action="append", default=[], metavar="KEY=VAL", help="bgv_cfg override for every context")
    args = ap.parse_args()
    cfg = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in args.cfg}
    import numpy as np
    import torch

    import bench
    from lodestar_amd import native

    dev = torch.device("cuda", 0)
    seg = bench.build_segment(list(range(args.blocks)))
    ctxs, arrs = [], []
    for k in range(args.ctx):
        d = native.Device(0, **cfg)
        d.gen_keys(0, bench.N_VALIDATORS, bench.SEED)
        da = bench.to_device(seg, torch, dev)
        sigs = torch.zeros((seg["n_sets"], 192), dtype=torch.uint8, device=dev)
        d.gen_sign(da, sigs, on_device=True)
        da.update(sigs=sigs, sig_len=torch.full((seg["n_sets"],), 96, dtype=torch.int32, device=dev), scalars=None)
        jr, _ = d.verify(da, on_device=True, want_set_codes=False)
        assert (jr == 1).all()
        ctxs.append(d)
        arrs.append(da)
    torch.cuda.synchronize()
    # back to back on context 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        jr, _ = ctxs[0].verify(arrs[0], on_device=True, want_set_codes=False)
    seq = (time.perf_counter() - t0) / args.steps * 1e3
    print(json.dumps({"mode": "sequential", "ms_per_batch": round(seq, 3)}), flush=True)
    # all contexts at once, one thread each
    oks = [True] * args.ctx

    def run(k):
        for _ in range(args.steps):
            jr, _ = ctxs[k].verify(arrs[k], on_device=True, want_set_codes=False)
            oks[k] &= bool((jr == 1).all())

    th = [threading.Thread(target=run, args=(k,)) for k in range(args.ctx)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    par = (time.perf_counter() - t0) / (args.steps * args.ctx) * 1e3
    print(json.dumps({"mode": f"{args.ctx} contexts in flight", "ms_per_batch": round(par, 3), "ok": all(oks),
                      "gain": round(seq / par, 4), "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                      **({"cfg": cfg} if cfg else {})}), flush=True)
    for d in ctxs:
        d.close()


if __name__ == "__main__":
    main()
