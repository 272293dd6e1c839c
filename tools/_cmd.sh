#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=r05zw
timeout -k 10 500 tools/ab.sh "base smp5" 3 --scene sphere_box_conductor --fpl 128 --spp 128 > gpurun_out/${T}_ab_smp5_c3.log 2>&1 || exit 1
timeout -k 10 500 tools/ab.sh "base smp5" 2 --scene sponza_class --fpl 128 --spp 128 > gpurun_out/${T}_ab_smp5_c5.log 2>&1 || exit 1
timeout -k 10 500 tools/ab.sh "base smp5" 2 --scene sphere_box_layered --fpl 128 --spp 128 > gpurun_out/${T}_ab_smp5_4l.log 2>&1 || exit 1
for c in c3 c5 4l; do python3 tools/ab_summary.py gpurun_out/${T}_ab_smp5_$c.log; done
