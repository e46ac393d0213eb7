"""Kernel-level view of batches in flight (tools/inflight_trace.py TRACE.csv):
over the window of the last N k_batch_final dispatches of a rocprofv3 kernel
trace of `bench.py --no-c2 --no-cpu` (C4 batches, several in flight), print
  * the window, batches finished in it and ms per batch;
  * the time with at least one kernel resident, and the mean number of
    resident dispatches (a concurrency measure);
  * per kernel: dispatches, mean duration, and its summed duration per batch
    (dispatch time, overlapping other kernels).
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--batches", type=int, default=16)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows]
    ev.sort()
    fin = sorted(e for _, e, k in ev if k.endswith("k_batch_final"))
    assert len(fin) > args.batches + 1, "too few batches in the trace"
    t0, t1 = fin[-args.batches - 1], fin[-1]
    win = [(max(s, t0), min(e, t1), k) for s, e, k in ev if e > t0 and s < t1]
    # union of busy time and mean residency
    pts = sorted([(s, 1) for s, _, _ in win] + [(e, -1) for _, e, _ in win])
    busy = area = 0
    cur, last = 0, t0
    for t, d in pts:
        if cur > 0:
            busy += t - last
        area += cur * (t - last)
        cur += d
        last = t
    span = t1 - t0
    print(f"window {span / 1e6:.3f} ms, {args.batches} batches: {span / 1e6 / args.batches:.3f} ms per batch")
    print(f"some kernel resident {busy / span:.4f} of the window; mean resident dispatches {area / span:.2f}")
    per = defaultdict(lambda: [0, 0])
    for s, e, k in win:
        per[k][0] += 1
        per[k][1] += e - s
    print(f"{'kernel':28s} {'disp/batch':>10s} {'mean ms':>9s} {'ms/batch':>9s}")
    for k, (n, tot) in sorted(per.items(), key=lambda x: -x[1][1]):
        if tot / span < 0.002:
            continue
        print(f"{k:28s} {n / args.batches:10.2f} {tot / n / 1e6:9.3f} {tot / 1e6 / args.batches:9.3f}")


if __name__ == "__main__":
    main()
