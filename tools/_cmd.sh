#!/bin/bash
# ad-hoc GPU step (see git log for what each call measured)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "sah or degenerate or bitexact or sponza" tests > gpurun_out/r04v_gputest_reinsert_undo.log 2>&1 && \
tools/ab.sh "noreins reins" 3 --scene sponza_class > gpurun_out/r04v_ab_reinsert_undo_sponza.log 2>&1
