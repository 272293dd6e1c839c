#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=r05o
timeout -k 10 1000 tools/ab.sh "base ntq" 4 --scene sphere_box_diffuse --fpl 64 --spp 128 --modes 1,2,3 > gpurun_out/${T}_ab_ntq.log 2>&1 || exit 1
python3 tools/ab_summary.py gpurun_out/${T}_ab_ntq.log
