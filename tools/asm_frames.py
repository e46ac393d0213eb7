"""Per-function register and scratch use of a gfx950 assembly file (hipcc
-save-temps), demangled: `python3 tools/asm_frames.py X-hip-amdgcn-amd-amdhsa-gfx950.s`."""
import re
import subprocess
import sys

cur = None
rows = {}
for line in open(sys.argv[1]):
    m = re.match(r"^(_Z\w+):", line)
    if m:
        cur = m.group(1)
        rows.setdefault(cur, {})
        continue
    m = re.match(r"^\s*;\s*(NumVgprs|NumAgprs|ScratchSize|Occupancy|TotalNumVgprs):\s*(\d+)", line)
    if m and cur:
        rows[cur][m.group(1)] = int(m.group(2))
names = list(rows)
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
for n, d in zip(names, dem):
    r = rows[n]
    if not r:
        continue
    d = re.sub(r"\(.*", "", d).replace("bgv::", "")
    print(f"{d[:60]:60s} vgpr={r.get('NumVgprs', '?'):>3} agpr={r.get('NumAgprs', 0):>3} scratch={r.get('ScratchSize', '?'):>5}"
          + (f" occ={r['Occupancy']}" if "Occupancy" in r else ""))
