#!/bin/bash
# ad-hoc GPU step (see git log for what each call measured)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "sah or degenerate or bitexact" tests > gpurun_out/r04u_gputest_reinsert.log 2>&1 && \
tools/ab.sh "noreins reins" 3 --scene sponza_class > gpurun_out/r04u_ab_reinsert_sponza.log 2>&1 && \
tools/ab.sh "noreins reins" 2 --scene sphere_box_diffuse --modes 3 >> gpurun_out/r04u_ab_reinsert_sponza.log 2>&1
