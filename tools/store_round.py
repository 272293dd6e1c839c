#!/usr/bin/env python3
"""Copy a tools/round.sh TAG run from gpurun_out/ into profiles/ and refresh the derived files.

    python tools/store_round.py TAG profile   after `tools/round.sh TAG profile` (run first)
    python tools/store_round.py TAG bench     after `tools/round.sh TAG bench`
profile: the rocprofv3 kernel stats (two-stream and one-stream passes, and configs 3 and 5) and
the PMC traces; writes profiles/traffic.json, profiles/shade_pmc.json (tools/shade_pmc.py over
the one-stream kernel stats), valu.json, vmem.json and shade_valu_config*.json, which the bench
lines then report as figures of their own sources.  bench: the bench JSONs of every config and
the GPU-test log.
"""
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def main():
    tag = sys.argv[1]
    part = sys.argv[2] if len(sys.argv) > 2 else "profile"
    prof, rnd, out = ROOT / "gpurun_out" / f"prof_{tag}", ROOT / "gpurun_out" / f"round_{tag}", ROOT / "profiles"
    if part == "bench":
        cp = [(rnd / "gputest.log", f"{tag}_gputest.log")]
        cp += [(rnd / f"bench_config{c}.json", f"{tag}_bench_config{c}.json") for c in ("2", "3", "4l", "5", "5t", "4d")]
        for src, dst in cp:
            shutil.copyfile(src, out / dst)
        return
    cp = [(prof / "kt" / "run_kernel_stats.csv", f"{tag}_wavefront_kernel_stats.csv"),
          (prof / "kt1" / "run_kernel_stats.csv", f"{tag}_wavefront_kernel_stats_single_stream.csv"),
          (prof / "fetch" / "run_counter_collection.csv", f"{tag}_wavefront_pmc_fetch_trace.csv"),
          (prof / "write" / "run_counter_collection.csv", f"{tag}_wavefront_pmc_write_trace.csv"),
          (prof / "traffic.json", f"{tag}_wavefront_traffic.json"),
          (prof / "traffic.json", "traffic.json")]
    cp += [(rnd / f"kt_config{c}" / "run_kernel_stats.csv", f"{tag}_kernel_stats_config{c}.csv") for c in ("3", "5")
           if (rnd / f"kt_config{c}" / "run_kernel_stats.csv").exists()]
    cp += [(rnd / f"kt1_config{c}" / "run_kernel_stats.csv", f"{tag}_kernel_stats_config{c}_single_stream.csv")
           for c in ("3", "5") if (rnd / f"kt1_config{c}" / "run_kernel_stats.csv").exists()]
    for src, dst in cp:
        shutil.copyfile(src, out / dst)
    pmc = subprocess.run([sys.executable, str(ROOT / "tools" / "shade_pmc.py"),
                          str(out / f"{tag}_wavefront_pmc_fetch_trace.csv"), str(out / f"{tag}_wavefront_pmc_write_trace.csv"),
                          str(out / f"{tag}_wavefront_kernel_stats_single_stream.csv")],
                         check=True, capture_output=True, text=True).stdout
    (out / "shade_pmc.json").write_text(pmc)
    # SQ / TCC / TCP and TA / TD passes of k_trace_pair (roofline.valu_pmc / vmem_pmc) and the
    # k_shade_nee VALU passes of the Default / Layered configs (roofline.valu)
    summ = ROOT / "tools" / "pmc_summary.py"
    if (ROOT / "gpurun_out" / f"pmc_{tag}").exists():
        txt = subprocess.run([sys.executable, str(summ), str(ROOT / "gpurun_out" / f"pmc_{tag}"), "k_trace_pair",
                              "--valu-json", str(out / "valu.json"), "--waves", "6",
                              "--source", f"tools/round.sh {tag} profile (tools/pmc.sh, Lambert, 64 frames)"],
                             check=True, capture_output=True, text=True).stdout
        (out / f"{tag}_pmc_trace_pair_lambert.txt").write_text(txt)
    if (ROOT / "gpurun_out" / f"pmcta_{tag}").exists():
        txt = subprocess.run([sys.executable, str(summ), str(ROOT / "gpurun_out" / f"pmcta_{tag}"), "k_trace_pair",
                              "--vmem-json", str(out / "vmem.json"),
                              "--source", f"tools/round.sh {tag} profile (tools/pmc_ta.sh, Lambert, 64 frames)"],
                             check=True, capture_output=True, text=True).stdout
        (out / f"{tag}_pmc_ta_td_trace_pair.txt").write_text(txt)
    for c in ("3", "4l", "5"):
        src = rnd / f"shade_valu_config{c}.json"
        if src.exists():
            shutil.copyfile(src, out / f"shade_valu_config{c}.json")


if __name__ == "__main__":
    main()
