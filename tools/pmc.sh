#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over tools/perf_probe.py, run from the
# repo root on the GPU box.  Summarise with tools/pmc_summary.py OUTDIR KERNEL_SUBSTRING.
#   tools/pmc.sh OUTDIR [perf_probe args...]
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
ARGS="$@"
ROOT="$GRAFT_REPO_ROOT"; [ -z "$ROOT" ] && ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && mkdir -p "$OUT"
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 tools/perf_probe.py --spp 8 --repeat 1 $ARGS > "$OUT/$name.log" 2>&1
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sq2 SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR
run tcc TCC_HIT_sum TCC_MISS_sum
run tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum
echo pmc-done
