#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r05w_gputest.log 2>&1; rc=$?; tail -3 gpurun_out/r05w_gputest.log; exit $rc
