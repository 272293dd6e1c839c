#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
PTAMD_LIB=optixpathtracer_amd/_variants/lib_tail.so timeout -k 10 300 python3 tools/perf_probe.py --scene sphere_box_diffuse --fpl 128 --spp 128 --repeat 1 --modes 1,3 > gpurun_out/r05zz_tail_final.log 2>&1 || exit 1
grep -c TAIL gpurun_out/r05zz_tail_final.log
