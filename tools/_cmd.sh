#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=r05zz
timeout -k 10 700 tools/ab.sh "base l512 l256" 3 --scene sphere_box_diffuse --fpl 128 --spp 256 --modes 1 > gpurun_out/${T}_ab_lblock.log 2>&1 || exit 1
python3 tools/ab_summary.py gpurun_out/${T}_ab_lblock.log
