#!/usr/bin/env python3
"""HBM traffic per launch of the dominant render kernel from rocprofv3 PMC passes.

    python tools/traffic.py PROFILE_DIR   (written by tools/profile.sh)

FETCH_SIZE and WRITE_SIZE come from separate rocprofv3 runs.  Both are in KiB.  On gfx950
FETCH_SIZE reports half the bytes of wide coalesced reads (MI355X_MICROARCH.md §HBM), so
`hbm_bytes_per_launch` doubles it.  The calibration of tools/hbm_calib.hip
(profiles/r02_hbm_calib.json) confirms the half count for streamed 16-B-per-lane reads and for
runs of 24 records, but shows a random 16-B gather counted at 4x its payload (a line fetch per
gather) with no evidence for doubling it, and WRITE_SIZE exact for streamed and window-shuffled
16-B stores but 2x for random 16-B stores (32-B write granule).  The trace kernels mix streamed
queue reads with gathers (W.L adds, BVH lines refetched from the Infinity Cache), so
`hbm_bytes_per_launch_low` = FETCH_SIZE + WRITE_SIZE is reported beside it: the HBM bytes lie
between the two.  The result is written to profiles/traffic.json, where bench.py reads it for
`roofline.traffic` / `roofline.traffic_low`.
"""
from __future__ import annotations

import csv
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from optixpathtracer_amd.provenance import kernel_sources_sha  # noqa: E402

# dominant kernels, per kernel: the megakernel, the fused modes'
# k_trace_pair, the Default / Layered modes' k_shade_nee
GROUPS = {"k_render_mega": ("k_render_mega",), "k_trace_pair": ("k_trace_pair",), "k_shade_nee": ("k_shade_nee",)}


def timed_instance(name: str) -> bool:
    """The kernels bench.py times: not the traversal-statistics instances (template STATS = true,
    bench.py's untimed counter render), whose counter atomics add writes of their own."""
    return "<true" not in name


def counter_rows(d: Path):
    for f in sorted(d.rglob("*counter_collection.csv")):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def per_kernel(d: Path, counter: str):
    vals: dict[str, list[float]] = {}
    for row in counter_rows(d):
        if row.get("Counter_Name") != counter:
            continue
        name = row["Kernel_Name"]
        if not timed_instance(name):
            continue
        for g, members in GROUPS.items():
            if any(k in name for k in members):
                vals.setdefault(g, []).append(float(row["Counter_Value"]))
    return vals


def kernel_stats(d: Path):
    out = {}
    for f in sorted(d.rglob("*kernel_stats.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if not timed_instance(row["Name"]):
                    continue
                for g, members in GROUPS.items():
                    if any(k in row["Name"] for k in members):
                        o = out.setdefault(g, {"calls": 0, "total_ns": 0.0})
                        o["calls"] += int(row["Calls"])
                        o["total_ns"] += float(row["TotalDurationNs"])
    for o in out.values():
        o["avg_ns"] = o["total_ns"] / max(1, o["calls"])
    return out


def main():
    root = Path(sys.argv[1])
    fetch = per_kernel(root / "fetch", "FETCH_SIZE")
    write = per_kernel(root / "write", "WRITE_SIZE")
    stats = kernel_stats(root / "kt")
    kernel = next((k for k in GROUPS if k in fetch and k in write), None)
    if kernel is None:
        print(json.dumps({"error": "no PMC rows for the render kernels"}))
        return
    f_kib = sum(fetch[kernel]) / len(fetch[kernel])
    w_kib = sum(write[kernel]) / len(write[kernel])
    hbm = 2.0 * f_kib * 1024.0 + w_kib * 1024.0
    low = f_kib * 1024.0 + w_kib * 1024.0
    # read requests by size (tools/profile.sh `rdsz` pass): the read bytes without the half-count
    # question -- k_trace_pair's are all 128-B requests (profiles/r05n_*), FETCH_SIZE tallies 64 B each
    sizes = None
    if (root / "rdsz").exists():
        n = {c: per_kernel(root / "rdsz", c).get(kernel) for c in
             ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")}
        if all(n.values()):
            m = {c: sum(v) / len(v) for c, v in n.items()}
            rd = 32 * m["TCC_EA0_RDREQ_32B_sum"] + 64 * m["TCC_EA0_RDREQ_64B_sum"] + 128 * m["TCC_EA0_RDREQ_128B_sum"]
            sizes = {"read_requests": round(m["TCC_EA0_RDREQ_sum"]), "of_them_128b": round(m["TCC_EA0_RDREQ_128B_sum"]),
                     "of_them_64b": round(m["TCC_EA0_RDREQ_64B_sum"]), "of_them_32b": round(m["TCC_EA0_RDREQ_32B_sum"]),
                     "read_bytes": int(rd), "hbm_bytes_per_launch_by_request_size": int(rd + w_kib * 1024.0)}
    print(json.dumps({
        "kernel": kernel,
        "dispatches": len(fetch[kernel]),
        "fetch_size_kib_mean": round(f_kib, 3),
        "write_size_kib_mean": round(w_kib, 3),
        "hbm_bytes_per_launch": int(hbm),
        "hbm_bytes_per_launch_low": int(low),
        "read_request_sizes": sizes,
        "kernel_trace": stats.get(kernel),
        # the same bench on one wavefront stream (tools/profile.sh kt1): solo launch times
        "kernel_trace_single_stream": kernel_stats(root / "kt1").get(kernel) if (root / "kt1").exists() else None,
        # the kernel sources these passes ran (bench.py reports the figures only on the same sources)
        "sources_sha": kernel_sources_sha(),
        "correction": "2 x FETCH_SIZE (gfx950 half-count) + WRITE_SIZE, KiB -> bytes; low: FETCH_SIZE + "
                      "WRITE_SIZE (a lower bound only: read_request_sizes counts the requests by size, and "
                      "where all are 128-B lines the first figure is exact)",
    }, indent=1))


if __name__ == "__main__":
    main()
