#!/usr/bin/env python3
"""Summarise tools/pmc.sh output for one kernel: per-dispatch means and derived ratios.

    python tools/pmc_summary.py OUTDIR KERNEL_SUBSTRING
"""
import csv
import sys
from collections import defaultdict
from pathlib import Path


def main():
    root, kname = Path(sys.argv[1]), sys.argv[2]
    acc = defaultdict(list)
    for f in root.rglob("*counter_collection.csv"):
        for row in csv.DictReader(open(f)):
            if kname in row["Kernel_Name"]:
                acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in acc.items()}
    for k in sorted(m):
        print(f"{k:24s} {m[k]:16.1f}  (n={len(acc[k])})")
    g = m.get
    if g("SQ_ACTIVE_INST_VALU") and g("SQ_THREAD_CYCLES_VALU"):
        print(f"VALU lane utilisation      {g('SQ_THREAD_CYCLES_VALU') / (64 * g('SQ_ACTIVE_INST_VALU')):.3f}")
    if g("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if g(k):
                print(f"{k:24s} / wave cycles  {g(k) / g('SQ_WAVE_CYCLES'):.3f}")
    if g("SQ_INSTS_VALU"):
        for k in ("SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_BRANCH"):
            if g(k):
                print(f"{k:24s} / VALU insts   {g(k) / g('SQ_INSTS_VALU'):.3f}")
    if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum") is not None:
        print(f"L2 hit rate                {g('TCC_HIT_sum') / max(1.0, g('TCC_HIT_sum') + g('TCC_MISS_sum')):.4f}")


if __name__ == "__main__":
    main()
