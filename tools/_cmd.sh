#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05f}
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${T}_gputest.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_gputest.log; exit $rc
