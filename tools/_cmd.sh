#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_counters.py > gpurun_out/r05s_counters.log 2>&1; rc=$?; tail -6 gpurun_out/r05s_counters.log; exit $rc
