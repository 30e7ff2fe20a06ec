"""Summarise a rocprofv3 kernel_stats.csv: top kernels, per-step totals."""
import csv, sys
path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
calls = sum(int(r['Calls']) for r in rows)
print(f"total GPU kernel time {tot/1e6:.3f} ms, {calls} dispatches; per step ({steps}): {tot/1e6/steps:.3f} ms, {calls/steps:.0f} kernels")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.3f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:8.2f}us {float(r['Percentage']):5.1f}%  {r['Name'][:100]}")
