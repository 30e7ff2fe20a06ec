"""Print the kernel sequence of the last training step in a rocprofv3 kernel trace
(a step is delimited by the fused AdamW kernel).  Usage: trace_step.py trace.csv [marker]"""
import csv, sys
from collections import Counter
rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else "adamw"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a, b = ends[-2] + 1, ends[-1] + 1
step = rows[a:b]
t0 = int(step[0]["Start_Timestamp"]); t1 = int(step[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
print(f"last step: {len(step)} kernels, wall {(t1-t0)/1e3:.1f} us, busy {busy/1e3:.1f} us")
c = Counter(); tt = Counter()
for r in step:
    n = r["Kernel_Name"][:90]
    c[n] += 1; tt[n] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for n, v in tt.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40):
    print(f"{v/1e3:8.1f} us {c[n]:4d}x  {n}")
if "-v" in sys.argv:
    for r in step:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        print(f"{d/1e3:7.2f} grid={r['Grid_Size_X']:>8} wg={r['Workgroup_Size_X']:>4} {r['Kernel_Name'][:110]}")
