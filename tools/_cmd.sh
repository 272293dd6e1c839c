#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=r05zi
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/${T}_gputest.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_gputest.log; [ $rc = 0 ] || exit $rc
PTAMD_LIB=optixpathtracer_amd/_variants/lib_tail.so timeout -k 10 200 python3 tools/perf_probe.py --scene sphere_box_diffuse --fpl 64 --spp 128 --repeat 1 --modes 1,3 --streams 1 > gpurun_out/${T}_tail_pool60.log 2>&1 || exit 1
grep TAIL gpurun_out/${T}_tail_pool60.log | head -8
