#!/bin/bash
# A/B of libptamd.so variants (tools/build_variants.sh) on the GPU box, interleaved so clock
# drift hits every variant alike.  Run from the repo root:
#   tools/ab.sh "v1 v2 ..." ROUNDS [perf_probe args...]
VARS=$1; ROUNDS=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $ROUNDS); do
  for v in $VARS; do
    echo "== $v round $r"
    PTAMD_LIB=optixpathtracer_amd/_variants/lib_$v.so timeout -k 10 120 python3 tools/perf_probe.py "$@" || exit 1
  done
done
