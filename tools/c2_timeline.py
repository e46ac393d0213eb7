"""Kernel timeline of the last C2 call in a rocprofv3 kernel trace
(tools/c2_timeline.py TRACE.csv): every dispatch after the second-to-last
k_batch_final's end up to the last k_batch_final's end, relative to the first
of them, with the gaps between consecutive dispatches."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
bf = [r for r in rows if "k_batch_final" in r["Kernel_Name"]]
t_prev, t_end = int(bf[-2]["End_Timestamp"]), int(bf[-1]["End_Timestamp"])
sel = [r for r in rows if int(r["Start_Timestamp"]) > t_prev and int(r["End_Timestamp"]) <= t_end]
t0 = int(sel[0]["Start_Timestamp"])
last_end = t0
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} dur {(e - s) / 1e3:8.1f} gap {(s - last_end) / 1e3:7.1f} us "
          f"q{r['Queue_Id']} {r['Kernel_Name'][:40]:40s} grid={r['Grid_Size_X']}x{r.get('Grid_Size_Y', '')}")
    last_end = max(last_end, e)
print(f"device span {(t_end - t0) / 1e3:.1f} us")
