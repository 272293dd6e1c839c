#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=r05x
timeout -k 10 500 tools/ab.sh "old new" 3 --scene sphere_box_conductor --fpl 64 --spp 64 > gpurun_out/${T}_ab_ntx_c3.log 2>&1 || exit 1
timeout -k 10 500 tools/ab.sh "old new" 3 --scene sponza_class --fpl 64 --spp 64 > gpurun_out/${T}_ab_ntx_c5.log 2>&1 || exit 1
timeout -k 10 300 tools/ab.sh "old new" 2 --scene sphere_box_diffuse --fpl 64 --spp 64 --modes 1,3 > gpurun_out/${T}_ab_ntx_c2.log 2>&1 || exit 1
for c in c3 c5 c2; do python3 tools/ab_summary.py gpurun_out/${T}_ab_ntx_$c.log; done
