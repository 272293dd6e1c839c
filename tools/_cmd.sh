#!/bin/bash
# ad-hoc GPU step (see git log for what each call measured)
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05b}
timeout -k 10 120 python3 tools/cancel_probe.py > gpurun_out/${T}_cancel_lambert.log 2>&1; echo "rc=$?"; tail -2 gpurun_out/${T}_cancel_lambert.log
timeout -k 10 120 python3 tools/cancel_probe.py --scene sphere_box_conductor > gpurun_out/${T}_cancel_default.log 2>&1; echo "rc=$?"; tail -2 gpurun_out/${T}_cancel_default.log
tools/ab.sh "base fast" 2 --scene sphere_box_conductor --fpl 64 --spp 128 > gpurun_out/${T}_ab_conductor.log 2>&1 && \
tools/ab.sh "base fast" 2 --scene sphere_box_layered --fpl 64 --spp 128 > gpurun_out/${T}_ab_layered.log 2>&1 && \
tools/ab.sh "base fast" 2 --scene sponza_class --fpl 64 --spp 128 > gpurun_out/${T}_ab_sponza.log 2>&1 && \
tools/ab.sh "base fast" 2 --scene sphere_box_dielectric20 --fpl 64 --spp 128 > gpurun_out/${T}_ab_dielectric.log 2>&1 && \
tools/ab.sh "base fast" 2 --scene sphere_box_diffuse --fpl 64 --spp 128 --modes 1,2 > gpurun_out/${T}_ab_diffuse.log 2>&1
