"""Per-kernel roofline table from the rocprofv3 passes written by tools/gpu_pmc_top.sh.

Usage: python tools/pmc_roofline.py <dir with pass sub-directories A/, B/, C/>

For the kernels that take the most time (kernel trace of pass A) it prints per dispatch:
  us        mean duration
  clk       effective clock GRBM_GUI_ACTIVE / 8 XCDs / duration (GHz)
  mfma%     SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel cycles): matrix-pipe utilisation
  valu%     SQ_ACTIVE_INST_VALU x 4 / (1024 x kernel cycles): vector issue share
  inst/wait shares of SQ_WAVE_CYCLES: ACTIVE_INST_ANY (issuing), WAIT_INST_ANY (issue
            stall: MFMA/VALU dependency, pipe busy), WAIT_ANY (parked on s_waitcnt/barrier)
  GB/s      (TCC_EA0_RDREQ + TCC_EA0_WRREQ) x 64 B / duration (HBM-side traffic, approx.)
and a one-word bound: "mfma" (matrix pipe >= 60 %), "hbm" (>= 3 TB/s), "issue" (issuing
>= 50 % of wave cycles), "latency" (waits dominate) or "launch" (< 4 us).
"""
import csv
import glob
import os
import sys
from collections import defaultdict

SIMDS = 1024


def _load_counters(d):
    acc = defaultdict(lambda: defaultdict(float))
    nd = defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "?")
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
            nd[k].add(row.get("Dispatch_Id", ""))
    return {k: {c: v / max(len(nd[k]), 1) for c, v in cs.items()} for k, cs in acc.items()}


def _load_durations(d):
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace*.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "?")
            tot[k] += (float(row["End_Timestamp"]) - float(row["Start_Timestamp"])) * 1e-3
            cnt[k] += 1
    return tot, cnt


def short(k, n=60):
    k = k.replace("void ", "").replace("hy::", "")
    i = k.find("(")
    return (k[:i] if i > 0 else k)[:n]


def main(d, top=14):
    tot, cnt = _load_durations(os.path.join(d, "A"))
    ctr = {}
    for p in ("A", "B", "C"):
        for k, cs in _load_counters(os.path.join(d, p)).items():
            ctr.setdefault(k, {}).update(cs)
    names = sorted(tot, key=lambda k: -tot[k])[:top]
    hdr = f"{'kernel':60s} {'us':>7s} {'clk':>5s} {'mfma%':>6s} {'valu%':>6s} {'inst%':>6s} {'stall%':>6s} {'wait%':>6s} {'GB/s':>7s} {'L2hit':>6s}  bound"
    print(hdr)
    for k in names:
        us = tot[k] / max(cnt[k], 1)
        c = ctr.get(k, {})
        clk = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0 / (us * 1e-6) / 1e9 if us > 0 else 0.0
        cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        mf = 100.0 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (SIMDS * cyc) if cyc else 0.0
        va = 100.0 * 4 * c.get("SQ_ACTIVE_INST_VALU", 0.0) / (SIMDS * cyc) if cyc else 0.0
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        ia = 100.0 * c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc if wc else 0.0
        st = 100.0 * c.get("SQ_WAIT_INST_ANY", 0.0) / wc if wc else 0.0
        wt = 100.0 * c.get("SQ_WAIT_ANY", 0.0) / wc if wc else 0.0
        by = 64.0 * (c.get("TCC_EA0_RDREQ_sum", 0.0) + c.get("TCC_EA0_WRREQ_sum", 0.0))
        gbs = by / (us * 1e-6) / 1e9 if us > 0 else 0.0
        # L2 hit rate needs BOTH counters of the same pass (TCC_MISS_sum was missing before
        # round 5, which printed a constant 100 %): report n/a rather than a fake rate
        h, m = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        l2 = 100.0 * h / (h + m) if (h is not None and m is not None and h + m > 0) else float("nan")
        if us < 4:
            b = "launch"
        elif mf >= 60:
            b = "mfma"
        elif gbs >= 3000:
            b = "hbm"
        elif ia >= 50:
            b = "issue"
        else:
            b = "latency"
        print(f"{short(k):60s} {us:7.1f} {clk:5.2f} {mf:6.1f} {va:6.1f} {ia:6.1f} {st:6.1f} {wt:6.1f} {gbs:7.0f} {l2:6.1f}  {b}")
    print("\nraw counters per dispatch:")
    for k in names:
        print(short(k, 90), f"(dispatches {cnt[k]})")
        for cn, v in sorted(ctr.get(k, {}).items()):
            print(f"   {cn:28s} {v:16.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
