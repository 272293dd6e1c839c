#!/bin/bash
# Where k_trace_pair's memory traffic goes: PMC passes over
# tools/perf_probe.py (Lambert, 1080p, 64 frames per batch) for libptamd variants, one rocprofv3 run
# per counter group, plus a traversal-statistics run for the per-launch ray counts.
#   tools/traffic_classes.sh OUTDIR "base noadd ntq"    (SIZES_ONLY=1: the read-request size pass alone)
set -e
OUT=${1:-gpurun_out/tc}; VARS=${2:-base}
ROOT="$GRAFT_REPO_ROOT"; [ -z "$ROOT" ] && ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && mkdir -p "$OUT"
timeout -k 10 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
for v in $VARS; do
  if [ "$v" = base ]; then L="$ROOT/optixpathtracer_amd/libptamd.so"; else L="$ROOT/optixpathtracer_amd/_variants/lib_$v.so"; fi
  export PTAMD_LIB="$L"
  run() {  # name counters...
    local name=$1; shift
    timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/${v}_$name" -o run -- python3 tools/perf_probe.py --repeat 1 --fpl 64 --spp 64 > "$OUT/${v}_$name.log" 2>&1
  }
  if [ -n "$SIZES_ONLY" ]; then run tccsz TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_sum; echo "$v done"; continue; fi
  timeout -k 10 240 python3 tools/perf_probe.py --repeat 1 --fpl 64 --spp 64 --stats > "$OUT/${v}_stats.log" 2>&1
  run fetch FETCH_SIZE
  run write WRITE_SIZE
  run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
  run tccw TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
  run tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum
  echo "$v done"
done
