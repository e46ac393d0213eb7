"""Probe: the Node/Python pools' device 0 on a multi-device node: three bulk
contexts with bgv_cfg.cu_split = -32 (CU-masked streams: each takes a hardware
queue of its own, with its own scratch) verifying C4 batches at once, beside
a cu_split = +32 priority context verifying single blocks.  Prints one JSON
line; a queue-resource failure aborts the process.
    python tools/reserved_pool_probe.py [--ctx 3] [--cu 32] [--steps 4]"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=3)
    ap.add_argument("--cu", type=int, default=32)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--blocks", type=int, default=1024)
    ap.add_argument("--prio-sets", type=int, default=1, help="sets per priority call: 1 (verifyOnMainThread) or a block's 98")
    ap.add_argument("--gap-ms", type=float, default=0.0, help="idle time between priority calls")
    args = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from lodestar_amd import native

    dev = torch.device("cuda", 0)
    seg = bench.build_segment(list(range(args.blocks)))
    bulk = []
    for _ in range(args.ctx):
        d = native.Device(0, cu_split=-args.cu)
        d.gen_keys(0, bench.N_VALIDATORS, bench.SEED)
        bulk.append(d)
    prio = native.Device(0, cu_split=args.cu)
    prio.gen_keys(0, bench.N_VALIDATORS, bench.SEED)
    da = bench.to_device(seg, torch, dev)
    sigs = torch.zeros((seg["n_sets"], 192), dtype=torch.uint8, device=dev)
    (bulk[0] if bulk else prio).gen_sign(da, sigs, on_device=True)
    da.update(sigs=sigs, sig_len=torch.full((seg["n_sets"],), 96, dtype=torch.int32, device=dev), scalars=None)
    blk = bench.build_segment([0])
    if args.prio_sets == 1:  # the block's last set: a single-pubkey set, as a proposer signature
        blk = dict(blk, n_sets=1, n_jobs=1, job_offsets=np.array([0, 1], np.uint32),
                   pk_offsets=np.array([0, 1], np.uint32), pk_indices=blk["pk_indices"][-1:].copy(),
                   msgs=blk["msgs"][-1:].copy())
    one = bench.to_device(blk, torch, dev)
    s1 = torch.zeros((one["n_sets"], 192), dtype=torch.uint8, device=dev)
    prio.gen_sign(one, s1, on_device=True)
    one.update(sigs=s1, sig_len=torch.full((one["n_sets"],), 96, dtype=torch.int32, device=dev), scalars=None)
    torch.cuda.synchronize()
    # the priority call takes host arrays, as the pools' verifyOnMainThread path
    # does (the library stages them on its own streams; an on-device call would
    # first synchronise torch's stream, which shares a hardware queue with the
    # bulk streams)
    one = dict(blk, sigs=s1.cpu().numpy(), sig_len=np.full(blk["n_sets"], 96, np.uint32), scalars=None)
    oks = [True] * args.ctx
    stop = threading.Event()
    prio_ms = []

    def run(k):
        for _ in range(args.steps):
            jr, _ = bulk[k].verify(da, on_device=True, want_set_codes=False)
            oks[k] &= bool((jr == 1).all())

    def run_prio():
        while not stop.is_set() and (args.ctx or len(prio_ms) < 20):
            t = time.perf_counter()
            jr, _ = prio.verify(one, on_device=False, want_set_codes=False)
            prio_ms.append((time.perf_counter() - t) * 1e3)
            oks.append(bool((jr == 1).all()))
            if args.gap_ms:
                stop.wait(args.gap_ms / 1e3)

    th = [threading.Thread(target=run, args=(k,)) for k in range(args.ctx)]
    tp = threading.Thread(target=run_prio)
    t0 = time.perf_counter()
    tp.start()
    for t in th:
        t.start()
    for t in th:
        t.join()
    stop.set()
    tp.join()
    el = time.perf_counter() - t0
    prio_ms.sort()
    print(json.dumps({"bulk_contexts": args.ctx, "prio_sets": int(one["n_sets"]), "cu_split": -args.cu, "priority_cu": args.cu, "ok": all(oks),
                      "bulk_ms_per_batch": round(el * 1e3 / (args.ctx * args.steps), 3) if args.ctx else None,
                      "priority_calls": len(prio_ms), "priority_ms_p50": round(prio_ms[len(prio_ms) // 2], 3) if prio_ms else None,
                      "priority_ms_max": round(prio_ms[-1], 3) if prio_ms else None}), flush=True)
    for d in bulk + [prio]:
        d.close()


if __name__ == "__main__":
    main()
