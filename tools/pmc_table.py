"""Per-kernel table of rocprofv3 counter-collection CSVs (one or more --pmc
passes over the same command): for each kernel its largest-grid dispatch,
every counter collected, plus derived ratios when present.

    python tools/pmc_table.py PASS1.csv [PASS2.csv ...] [--kernels k_hash,k_miller]
"""
import csv
import sys
from collections import defaultdict


def load(paths):
    data = defaultdict(dict)  # (kernel, dispatch) -> counter -> value
    grid = {}
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("bgv::", "").replace("void ", "").strip()
            key = (k, int(r["Grid_Size"]))
            data[key][r["Counter_Name"]] = data[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            grid[key] = int(r["Grid_Size"])
    return data


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    want = None
    for a in sys.argv[1:]:
        if a.startswith("--kernels="):
            want = a.split("=", 1)[1].split(",")
    data = load(args)
    best = {}
    for (k, g), c in data.items():
        if want and k not in want:
            continue
        if k not in best or g > best[k][0]:
            best[k] = (g, c)
    for k, (g, c) in sorted(best.items(), key=lambda kv: -kv[1][1].get("SQ_WAVE_CYCLES", kv[1][1].get("SQ_BUSY_CYCLES", 0))):
        print(f"{k} grid={g}")
        for name in sorted(c):
            print(f"   {name:32s} {c[name]:16.0f}")
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if n in c:
                    print(f"   {n + ' / WAVE_CYCLES':32s} {c[n] / wc:16.3f}")
        if "SQC_ICACHE_REQ" in c and c["SQC_ICACHE_REQ"]:
            print(f"   {'icache miss rate':32s} {c.get('SQC_ICACHE_MISSES', 0) / c['SQC_ICACHE_REQ']:16.4f}")


if __name__ == "__main__":
    main()
