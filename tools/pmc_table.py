#!/usr/bin/env python3
"""Per-kernel PMC table from tools/gpu_pmc_diag.sh output (a/b/c_counters.csv): MFMA busy,
TD / TA / TCP stalls, L2 hit rate and latency, LDS activity, per dispatch averaged per kernel.

  python tools/pmc_table.py DIR [kernel-substring ...]
"""
import collections
import csv
import sys
from pathlib import Path

NCU, NXCD, NSIMD = 256, 8, 1024


def load(p):
    per = collections.defaultdict(lambda: collections.defaultdict(list))  # kernel -> counter -> [values per dispatch]
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(p)):
        disp[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    for (k, _), cs in disp.items():
        for c, v in cs.items():
            per[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}


def main():
    d = Path(sys.argv[1])
    pats = sys.argv[2:] or ["Li2E", "Li0ELi1", "coef_kernel"]
    m = {}
    for p in "abc":
        f = d / f"{p}_counters.csv"
        if f.exists():
            for k, cs in load(f).items():
                m.setdefault(k, {}).update(cs)
    for pat in pats:
        for k, c in m.items():
            if pat not in k:
                continue
            cyc = c.get("GRBM_GUI_ACTIVE", 0) / NXCD
            if cyc <= 0:
                continue
            row = {
                "cycles/XCD": f"{cyc / 1e3:.0f}k",
                "MFMA busy": f"{100 * c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (NSIMD * cyc):.0f} %" if 'SQ_VALU_MFMA_BUSY_CYCLES' in c else "-",
                "TD busy": f"{100 * c.get('TD_TD_BUSY_sum', 0) / NCU / cyc:.0f} %" if 'TD_TD_BUSY_sum' in c else "-",
                "TD stall on TCP": f"{100 * c.get('TD_TC_STALL_sum', 0) / NCU / cyc:.0f} %" if 'TD_TC_STALL_sum' in c else "-",
                "TCP pending stall": f"{100 * c.get('TCP_PENDING_STALL_CYCLES_sum', 0) / NCU / cyc:.0f} %" if 'TCP_PENDING_STALL_CYCLES_sum' in c else "-",
                "TA busy": f"{100 * c.get('TA_TA_BUSY_sum', 0) / NCU / cyc:.0f} %" if 'TA_TA_BUSY_sum' in c else "-",
                "L2 hit": (f"{100 * c['TCC_HIT_sum'] / (c['TCC_HIT_sum'] + c['TCC_MISS_sum']):.0f} %"
                           if c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0) > 0 else "-"),
                "L1->L2 latency": (f"{c['TCP_TCC_READ_REQ_LATENCY_sum'] / c['TCP_TCC_READ_REQ_sum']:.0f} cyc"
                                   if c.get("TCP_TCC_READ_REQ_sum", 0) > 0 else "-"),
                "LDS busy": f"{100 * c.get('SQ_LDS_IDX_ACTIVE', 0) / NCU / cyc:.0f} %" if 'SQ_LDS_IDX_ACTIVE' in c else "-",
                "LDS bank conflict": f"{c.get('SQ_LDS_BANK_CONFLICT', 0) / 1e3:.0f}k cyc" if 'SQ_LDS_BANK_CONFLICT' in c else "-",
            }
            print(f"## {k[:90]}")
            for a, b in row.items():
                print(f"| {a} | {b} |")


if __name__ == "__main__":
    main()
