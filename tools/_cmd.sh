#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 tools/traffic_classes.sh gpurun_out/r05l_tc "base noadd ntq"
