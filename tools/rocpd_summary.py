"""Summarise a rocprofv3 rocpd SQLite database (``*_results.db``).

Usage: python tools/rocpd_summary.py <db> [--last-fraction F] [--top K] [--steps S]

``--last-fraction`` keeps only dispatches in the final F of the kernel timeline
(e.g. the timed steps after warm-up); ``--steps`` divides totals to per-step.
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last-fraction", type=float, default=1.0)
    ap.add_argument("--last-ms", type=float, default=None, help="keep only the final MS of the timeline")
    ap.add_argument("--between", default=None,
                    help="keep only kernels between the last two dispatches whose name contains this (e.g. sleep)")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--sequence", type=int, default=0, help="print the last N dispatches in launch order")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    # workgroups of a dispatch over all three grid dimensions (grid sizes are in work-items)
    try:
        rows = list(c.execute("select name, start, end, grid_x * grid_y * grid_z, "
                              "workgroup_x * workgroup_y * workgroup_z, vgpr_count, accum_vgpr_count, lds_size "
                              "from kernels order by start"))
    except sqlite3.OperationalError:
        rows = list(c.execute("select name, start, end, grid_x, workgroup_x, vgpr_count, accum_vgpr_count, lds_size "
                              "from kernels order by start"))
    if not rows:
        print("no kernels")
        return
    t0, t1 = rows[0][1], max(r[2] for r in rows)
    cut = t1 - (t1 - t0) * a.last_fraction
    if a.last_ms is not None:
        cut = t1 - a.last_ms * 1e6
    rows = [r for r in rows if r[1] >= cut]
    if a.between:
        marks = [i for i, r in enumerate(rows) if a.between in r[0]]
        assert len(marks) >= 2, f"need two '{a.between}' marker kernels, found {len(marks)}"
        rows = rows[marks[-2] + 1:marks[-1]]
    if a.sequence:
        for name, s, e, gx, wx, vg, ag, lds in rows[-a.sequence:]:
            print(f"{(e - s) / 1e3:8.2f} us  wgs {gx // max(wx, 1):6d}  {name[:120]}")
        return
    agg = {}
    for name, s, e, gx, wx, vg, ag, lds in rows:
        d = agg.setdefault(name, [0, 0.0, gx // max(wx, 1), vg, ag, lds])
        d[0] += 1
        d[1] += (e - s)
    tot = sum(v[1] for v in agg.values())
    span = rows[-1][2] - rows[0][1]
    S = max(a.steps, 1)
    print(f"dispatches {len(rows)} ({len(rows) / S:.0f}/step)  kernel-busy {tot / 1e6:.3f} ms "
          f"({tot / 1e6 / S:.3f} ms/step)  timeline span {span / 1e6:.3f} ms ({span / 1e6 / S:.3f} ms/step)  "
          f"busy/span {100 * tot / max(span, 1):.1f}%")
    print(f"{'ms/step':>9} {'calls/st':>8} {'avg us':>8} {'%':>5} {'wgs':>6} {'vgpr':>5} {'agpr':>5} {'lds':>6}  kernel")
    for name, (n, d, wgs, vg, ag, lds) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{d / 1e6 / S:9.4f} {n / S:8.1f} {d / n / 1e3:8.2f} {100 * d / tot:5.1f} {wgs:6d} {vg:5d} {ag:5d} "
              f"{lds:6d}  {name[:110]}")


if __name__ == "__main__":
    main()
