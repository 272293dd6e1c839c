#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=r05zy
timeout -k 10 900 tools/ab.sh "base k1k k2k p80" 3 --scene sphere_box_diffuse --fpl 128 --spp 256 --modes 1,3 > gpurun_out/${T}_ab_pool128.log 2>&1 || exit 1
timeout -k 10 500 tools/ab.sh "base k1k k2k p80" 2 --scene sponza_class --fpl 128 --spp 128 > gpurun_out/${T}_ab_pool128_c5.log 2>&1 || exit 1
python3 tools/ab_summary.py gpurun_out/${T}_ab_pool128.log; python3 tools/ab_summary.py gpurun_out/${T}_ab_pool128_c5.log
