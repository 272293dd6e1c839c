"""Per-kernel PMC HBM bandwidth of the wavefront kernels from a tools/profile.sh run.

HBM bytes per launch = 2 x FETCH_SIZE (gfx950 half-count correction) + WRITE_SIZE, in KiB,
from the two separate --pmc passes; the average launch time comes from the kernel-trace pass
of the same batch size (64 frames per launch).  Writes profiles/shade_pmc.json, which bench.py
reports next to the trace-kernel roofline (k_shade_fused is the memory-bound kernel of a
Lambert frame).
    python tools/shade_pmc.py [fetch.csv write.csv kernel_stats.csv] > profiles/shade_pmc.json
(kernel_stats.csv: the one-stream pass, tools/profile.sh kt1 -- with two wavefront streams a
shading launch shares the GPU with the other stream's trace kernels and its time is not its own)
"""
import collections
import csv
import json
import re
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from optixpathtracer_amd.provenance import kernel_sources_sha  # noqa: E402

PEAK_GBPS = 8000.0


def name(n):
    m = re.search(r"(k_\w+(<[^>]*>)?)", n)
    return m.group(1) if m else n


def main():
    fetch, write, stats = (sys.argv[1:4] if len(sys.argv) >= 4 else
                           ("profiles/r01_wavefront_pmc_fetch_trace.csv", "profiles/r01_wavefront_pmc_write_trace.csv",
                            "profiles/r01_wavefront_kernel_stats.csv"))
    f, w = collections.defaultdict(list), collections.defaultdict(list)
    for fn, d in ((fetch, f), (write, w)):
        for r in csv.DictReader(open(fn)):
            d[name(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    avg = {name(r["Name"]): float(r["AverageNs"]) for r in csv.DictReader(open(stats))}
    out = {}
    for k in sorted(f):
        if not k.startswith(("k_shade", "k_trace", "k_extend", "k_shadow_vis")) or k not in avg or not w.get(k):
            continue
        b = (2.0 * sum(f[k]) / len(f[k]) + sum(w[k]) / len(w[k])) * 1024.0
        gbps = b / avg[k]
        out[k] = {"hbm_bytes_per_launch": int(b), "avg_launch_ms": round(avg[k] / 1e6, 4),
                  "hbm_gbps": round(gbps, 1), "frac": round(gbps / PEAK_GBPS, 4)}
    print(json.dumps({"kernels": out, "peak_gbps": PEAK_GBPS, "sources_sha": kernel_sources_sha(),
                      "correction": "2 x FETCH_SIZE (gfx950 half-count) + WRITE_SIZE, KiB -> bytes",
                      "sources": [fetch, write, stats]}, indent=1))


if __name__ == "__main__":
    main()
