"""Per-step timeline of a marked rocprofv3 trace (rocpd db): one line per dispatch with
start offset, duration, queue and the gap since the previous dispatch on the same queue,
plus per-queue busy totals.  Usage: python tools/step_timeline.py <db> [--step K]"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--step", type=int, default=5)
    ap.add_argument("--marker", default="spin_kernel")
    ap.add_argument("--first", default="assemble_kernel")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end, queue_id from kernels order by start"))
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    rows = rows[marks[-2] + 1:marks[-1]]
    starts = [i for i, r in enumerate(rows) if a.first in r[0]]
    i0, i1 = starts[a.step], starts[a.step + 1] if a.step + 1 < len(starts) else len(rows)
    step = rows[i0:i1]
    t0 = step[0][1]
    last = {}
    busy = {}
    for name, s, e, q in step:
        gap = (s - last[q]) / 1e3 if q in last else 0.0
        last[q] = e
        busy[q] = busy.get(q, 0) + (e - s)
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q % 100:<3d} gap{gap:6.1f}  {name[:90]}")
    span = (max(r[2] for r in step) - t0) / 1e3
    nxt = rows[i1][1] if i1 < len(rows) else None
    print(f"step span {span:.1f} us (to next step start {((nxt - t0) / 1e3) if nxt else float('nan'):.1f} us)")
    for q, b in busy.items():
        print(f"  queue {q}: busy {b / 1e3:.1f} us")


if __name__ == "__main__":
    main()
