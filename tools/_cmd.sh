#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
( timeout -k 10 200 python3 tools/build_probe.py --soup 1000000 --builders 4,3,1,2 --repeat 2 &&
  timeout -k 10 300 python3 tools/build_probe.py --soup 4000000 --builders 4,3,1 --repeat 2 ) > gpurun_out/r05y_build_soup.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/r05y_build_soup.log; exit $rc
