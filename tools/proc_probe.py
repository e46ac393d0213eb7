"""Probe: does a second PROCESS on the same GPU (its own four HIP hardware
queues) raise the in-flight throughput of small batches, where one process's
four queues cap the kernels running at once?  Each process opens --ctx
contexts, verifies --steps batches per context on one thread each, and
reports its own elapsed time; the processes start together (ready files).
    python tools/proc_probe.py --procs 2 --ctx 2 --blocks 128"""
import argparse
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(args):
    import torch

    import bench
    from lodestar_amd import native

    dev = torch.device("cuda", 0)
    seg = bench.build_segment(list(range(args.blocks)))
    ctxs, arrs = [], []
    for _ in range(args.ctx):
        d = native.Device(0)
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
    open(os.path.join(args.sync, f"ready_{os.getpid()}"), "w").close()
    while len([f for f in os.listdir(args.sync) if f.startswith("ready_")]) < args.procs:
        time.sleep(0.01)
    oks = [True] * args.ctx

    def run(k):
        for _ in range(args.steps):
            jr, _ = ctxs[k].verify(arrs[k], on_device=True, want_set_codes=False)
            oks[k] &= bool((jr == 1).all())

    th = [threading.Thread(target=run, args=(k,)) for k in range(args.ctx)]
    t0 = time.time()
    for t in th:
        t.start()
    for t in th:
        t.join()
    t1 = time.time()
    print(json.dumps({"pid": os.getpid(), "t0": t0, "t1": t1, "batches": args.steps * args.ctx, "ok": all(oks)}), flush=True)
    for d in ctxs:
        d.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--ctx", type=int, default=2)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--blocks", type=int, default=128)
    ap.add_argument("--sync", default="")
    ap.add_argument("--worker", action="store_true")
    args = ap.parse_args()
    if args.worker:
        return worker(args)
    sync = os.path.join(ROOT, "gpurun_out", f"proc_probe_sync_{os.getpid()}")
    os.makedirs(sync, exist_ok=True)
    cmd = [sys.executable, "-u", os.path.abspath(__file__), "--worker", "--procs", str(args.procs), "--ctx", str(args.ctx),
           "--steps", str(args.steps), "--blocks", str(args.blocks), "--sync", sync]
    ps = [subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True) for _ in range(args.procs)]
    outs = [json.loads(p.communicate()[0].strip().splitlines()[-1]) for p in ps]
    rc = max(p.returncode for p in ps)
    for f in os.listdir(sync):
        os.remove(os.path.join(sync, f))
    os.rmdir(sync)
    t0 = min(o["t0"] for o in outs)
    t1 = max(o["t1"] for o in outs)
    n = sum(o["batches"] for o in outs)
    print(json.dumps({"procs": args.procs, "ctx_per_proc": args.ctx, "blocks": args.blocks, "batches": n,
                      "ms_per_batch": round((t1 - t0) * 1e3 / n, 3), "ok": all(o["ok"] for o in outs),
                      "start_skew_ms": round((max(o["t0"] for o in outs) - t0) * 1e3, 2)}), flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main() or 0)
