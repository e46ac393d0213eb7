"""Fold two rocprofv3 counter-collection CSVs (one --pmc FETCH_SIZE pass, one
--pmc WRITE_SIZE pass, each over `bench.py --steps 1 --warmup 0 --no-c2
--no-cpu`) into tools/pmc_traffic.json: bytes per launch of each kernel.

    python tools/pmc_summary.py FETCH.csv WRITE.csv [--tag r01]

rocprofv3 reports both counters in KB; values are converted to bytes and left
raw (no gfx950 width correction: the dominant traffic is scratch, whose access
width is not the calibrated 16-B/lane streaming read of the microarch guide).
"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    """kernel -> (bytes of its largest-grid dispatch, number of dispatches)"""
    best, n = {}, defaultdict(int)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"].split("(")[0].replace("bgv::", "").strip()
            grid, val = int(row["Grid_Size"]), float(row["Counter_Value"]) * 1024.0
            n[name] += 1
            if name not in best or grid > best[name][0]:
                best[name] = (grid, val)
    return {k: v[1] for k, v in best.items()}, n


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    tag = sys.argv[sys.argv.index("--tag") + 1] if "--tag" in sys.argv else "r01"
    fetch, nf = per_kernel(args[0], "FETCH_SIZE")
    write, nw = per_kernel(args[1], "WRITE_SIZE")
    out = {
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), bench.py --steps 1 --warmup 0 --no-c2; "
                  f"profiles/{tag}_pmc_fetch_size.csv, profiles/{tag}_pmc_write_size.csv",
        "note": "per launch (the kernel's largest-grid dispatch); FETCH_SIZE is reported raw (KB x 1024): the gfx950 1/2 under-count the microarch guide documents "
                "for 16-B/lane streaming reads is NOT applied (these are scratch accesses, width uncalibrated)",
        "kernels": {},
    }
    for k in sorted(set(fetch) | set(write), key=lambda k: -(fetch.get(k, 0) + write.get(k, 0))):
        if not k.startswith("k_"):
            continue
        out["kernels"][k] = {"fetch_bytes": fetch.get(k, 0.0), "write_bytes": write.get(k, 0.0),
                             "dispatches": nf.get(k, 0), "dispatch": "largest grid"}
    with open(os.path.join(ROOT, "tools", "pmc_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    for k, v in list(out["kernels"].items())[:8]:
        print(f"{k:16s} fetch {v['fetch_bytes'] / 1e9:8.2f} GB  write {v['write_bytes'] / 1e9:8.2f} GB  ({v['dispatches']} dispatches)")


if __name__ == "__main__":
    main()
