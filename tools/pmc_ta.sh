#!/bin/bash
# Address/data-path PMC passes (TA, TD, TCP latency) over tools/perf_probe.py, GPU box, repo root.
#   tools/pmc_ta.sh OUTDIR [perf_probe args...]; summarise with tools/pmc_summary.py OUTDIR KERNEL
set -e
OUT=${1:-gpurun_out/pmc_ta}; shift || true
ARGS="$@"
ROOT="$GRAFT_REPO_ROOT"; [ -z "$ROOT" ] && ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && mkdir -p "$OUT"
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 tools/perf_probe.py --spp 8 --repeat 1 $ARGS > "$OUT/$name.log" 2>&1
}
run ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT
run td TD_TD_BUSY_sum TD_TC_STALL_sum
run tcp TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCP_LATENCY_sum
echo pmc-done
