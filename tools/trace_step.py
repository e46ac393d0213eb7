"""Print the kernel timeline of the last C4 step in a rocprofv3 kernel trace
(tools/trace_step.py TRACE.csv): start/end/duration per dispatch relative to
the end of the previous step's batch final exponentiation."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
km = [r for r in rows if "k_miller(" in r["Kernel_Name"]]
last = km[-1]
s0 = int(last["Start_Timestamp"])
bf = [r for r in rows if "k_batch_final" in r["Kernel_Name"]]
prev = [r for r in bf if int(r["End_Timestamp"]) < s0][-1]
nxt = [r for r in bf if int(r["Start_Timestamp"]) > s0][0]
t0, t1 = int(prev["End_Timestamp"]), int(nxt["End_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s >= t0 and e <= t1:
        print(f"{(s - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s) / 1e6:8.3f} q{r['Queue_Id']} {r['Kernel_Name'][:36]:36s} "
              f"grid={r['Grid_Size_X']} vgpr={r['VGPR_Count']}/{r['Accum_VGPR_Count']} lds={r['LDS_Block_Size']} scr={r['Scratch_Size']}")
print(f"step span {(t1 - t0) / 1e6:.3f} ms")
