#!/bin/bash
# PMC passes for the layered NEE kernel (k_shade_nee), one rocprofv3 run per counter group over
# tools/perf_probe.py, from the repo root on the GPU box: issue and wait cycles, instruction mix,
# instruction-fetch and instruction-cache counters, scratch traffic.  Summarise with
# tools/pmc_summary.py OUTDIR/<pass> k_shade_nee.
#   tools/pmc_shade.sh OUTDIR [perf_probe args...]
set -e
OUT=${1:-gpurun_out/pmc_shade}; shift || true
ARGS="$@"
ROOT="$GRAFT_REPO_ROOT"; [ -z "$ROOT" ] && ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && mkdir -p "$OUT"
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python3 tools/perf_probe.py --repeat 1 $ARGS > "$OUT/$name.log" 2>&1
  echo "pass $name done"
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sq2 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_IFETCH_LEVEL SQ_THREAD_CYCLES_VALU
run sqc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE
run sq3 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES SQ_INSTS_FLAT SQ_INSTS_VALU_TRANS_F32
echo pmc-shade-done
