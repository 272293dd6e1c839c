#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05k}
for v in s128 s64 s32; do
  L=optixpathtracer_amd/_variants/lib_$v.so
  echo "== $v"; PTAMD_LIB=$L timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sah_builder.py 2>&1 | tail -2 || exit 1
  PTAMD_LIB=$L timeout -k 10 200 python3 tools/build_probe.py --builders 4 --repeat 4 || exit 1
  PTAMD_LIB=$L timeout -k 10 200 python3 tools/build_probe.py --builders 4 --repeat 3 --scene sphere_box_diffuse || exit 1
done > gpurun_out/${T}_build_probe.log 2>&1
cd /tmp && export TMPDIR=/tmp && PTAMD_LIB=$GRAFT_REPO_ROOT/optixpathtracer_amd/_variants/lib_s64.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/build_probe.py --builders 4 --repeat 3 > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log 2>&1
