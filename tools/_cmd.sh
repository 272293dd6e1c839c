#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=r05zb
timeout -k 10 700 tools/ab.sh "trd0 cur" 4 --scene sphere_box_dielectric20 --fpl 64 --spp 128 > gpurun_out/${T}_ab_trd_4d.log 2>&1 || exit 1
timeout -k 10 700 tools/ab.sh "trd0 cur" 3 --scene sphere_box_layered --fpl 64 --spp 64 > gpurun_out/${T}_ab_trd_4l.log 2>&1 || exit 1
python3 tools/ab_summary.py gpurun_out/${T}_ab_trd_4d.log; python3 tools/ab_summary.py gpurun_out/${T}_ab_trd_4l.log
