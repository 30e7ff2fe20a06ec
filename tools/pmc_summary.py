"""Per-kernel totals of a rocprofv3 --pmc csv run directory (mean over dispatches).
Usage: python tools/pmc_summary.py <dir>"""
import csv
import glob
import sys
from collections import defaultdict


def main(d):
    files = glob.glob(f"{d}/**/*counter_collection*.csv", recursive=True)
    if not files:
        print("no counter csv under", d)
        return
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in files:
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "?")[:90]
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[k].add(row.get("Dispatch_Id", ""))
    for k, cs in acc.items():
        n = max(len(disp[k]), 1)
        print(k, f"(dispatches {n})")
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} {v / n:16.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
