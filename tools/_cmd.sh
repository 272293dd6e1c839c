#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=r05zm
timeout -k 10 1000 tools/ab.sh "base r12 r20 t16 t24" 3 --scene sphere_box_diffuse --fpl 64 --spp 128 --modes 1,3 > gpurun_out/${T}_ab_thresholds.log 2>&1 || exit 1
python3 tools/ab_summary.py gpurun_out/${T}_ab_thresholds.log
