#!/usr/bin/env python3
"""Summarise tools/pmc.sh output for one kernel: per-dispatch means and derived ratios.

    python tools/pmc_summary.py OUTDIR KERNEL_SUBSTRING [--valu-json OUT --waves N --source TEXT]
                                                        [--vmem-json OUT]

--valu-json writes the VALU figures bench.py reports as roofline.valu_pmc (profiles/valu.json),
tagged with the kernel sources they were measured on; --waves is the kernel's waves per SIMD.
--vmem-json writes the vector-memory figures of the tools/pmc_ta.sh passes (roofline.vmem_pmc,
profiles/vmem.json): the busy fraction of the per-CU texture address (TA) and data (TD) units,
the TD cycles stalled on the cache, and the mean L1 -> L2 read latency.  The TA/TD counters sum
over the 256 CUs and GRBM_GUI_ACTIVE over the 8 XCDs, so a unit's busy fraction is
(X_BUSY_sum / 256) / (GRBM_GUI_ACTIVE / 8).
SQ counters are per wave and count quad-cycles, so `valu_issue_slots` = issue fraction x resident
waves is the share of a SIMD's quad-cycles with a VALU issue.  With several waves a SIMD issues a
wave64 VALU instruction every 2 cycles (MI355X_MICROARCH.md, per-instruction cycle constants), two
per quad-cycle, so the VALU pipe is busy `valu_busy` = valu_issue_slots / 2 of the time (rounds
1-3 reported valu_issue_slots as the busy fraction).
"""
import argparse
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from optixpathtracer_amd.provenance import kernel_sources_sha  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("kernel")
    ap.add_argument("--valu-json", default=None)
    ap.add_argument("--waves", type=int, default=6)
    ap.add_argument("--source", default="")
    ap.add_argument("--vmem-json", default=None)
    ap.add_argument("--shade-json", default=None,
                    help="write the VALU figures of a shading kernel (k_shade_nee) that bench.py reports as "
                         "roofline.valu (profiles/shade_valu_config<C>.json)")
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--xcds", type=int, default=8)
    a = ap.parse_args()
    root, kname = Path(a.outdir), a.kernel
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
    if a.valu_json and g("SQ_ACTIVE_INST_VALU") and g("SQ_WAVE_CYCLES") and g("SQ_THREAD_CYCLES_VALU"):
        issue = g("SQ_ACTIVE_INST_VALU") / g("SQ_WAVE_CYCLES")
        Path(a.valu_json).write_text(json.dumps({
            "kernel": kname,
            "source": a.source or f"tools/pmc.sh -> {root}",
            "sources_sha": kernel_sources_sha(),
            "waves_per_simd": a.waves,
            "valu_issue_per_wave_cycle": round(issue, 3),
            "valu_issue_slots": round(min(1.0, issue * a.waves), 3),
            "valu_busy": round(min(1.0, issue * a.waves / 2.0), 3),
            "lane_utilisation": round(g("SQ_THREAD_CYCLES_VALU") / (64 * g("SQ_ACTIVE_INST_VALU")), 3),
            "wait_per_wave_cycle": round(g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"), 3) if g("SQ_WAIT_ANY") else None,
        }, indent=1) + "\n")
    if a.shade_json and g("SQ_INSTS_VALU") and g("SQ_ACTIVE_INST_VALU") and g("SQ_THREAD_CYCLES_VALU"):
        Path(a.shade_json).write_text(json.dumps({
            "kernel": kname,
            "source": a.source or f"tools/pmc.sh -> {root}",
            "sources_sha": kernel_sources_sha(),
            "dispatches": len(acc["SQ_INSTS_VALU"]),
            "valu_insts_per_dispatch": round(g("SQ_INSTS_VALU")),
            "lane_utilisation": round(g("SQ_THREAD_CYCLES_VALU") / (64 * g("SQ_ACTIVE_INST_VALU")), 3),
            "valu_issue_per_wave_cycle": round(g("SQ_ACTIVE_INST_VALU") / g("SQ_WAVE_CYCLES"), 3)
            if g("SQ_WAVE_CYCLES") else None,
            "wait_per_wave_cycle": round(g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"), 3)
            if g("SQ_WAIT_ANY") and g("SQ_WAVE_CYCLES") else None,
        }, indent=1) + "\n")
    if g("GRBM_GUI_ACTIVE") and g("TA_TA_BUSY_sum") and g("TD_TD_BUSY_sum"):
        cyc = g("GRBM_GUI_ACTIVE") / a.xcds  # per-XCD active cycles of the dispatch
        per = lambda k: round(g(k) / a.cus / cyc, 3) if g(k) is not None else None  # noqa: E731
        vm = {"ta_busy": per("TA_TA_BUSY_sum"), "td_busy": per("TD_TD_BUSY_sum"),
              "ta_stalled_by_tc": per("TA_ADDR_STALLED_BY_TC_CYCLES_sum"), "td_tc_stall": per("TD_TC_STALL_sum"),
              "l2_read_latency_cycles": round(g("TCP_TCC_READ_REQ_LATENCY_sum") / g("TCP_TCC_READ_REQ_sum"), 1)
              if g("TCP_TCC_READ_REQ_sum") else None}
        for k, v in vm.items():
            print(f"{k:24s} {v}")
        if a.vmem_json:
            Path(a.vmem_json).write_text(json.dumps({
                "kernel": kname, "source": a.source or f"tools/pmc_ta.sh -> {root}",
                "sources_sha": kernel_sources_sha(), **vm}, indent=1) + "\n")


if __name__ == "__main__":
    main()
