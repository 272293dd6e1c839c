#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the GPU box (repo root): tools/hbm_calib (built by
# hipcc from tools/hbm_calib.hip) under one rocprofv3 pass per counter, then tools/hbm_calib.py.
#   tools/hbm_calib.sh OUTDIR
set -e
OUT=${1:-gpurun_out/hbm_calib}
ROOT="$GRAFT_REPO_ROOT"; [ -z "$ROOT" ] && ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && mkdir -p "$OUT"
timeout -k 10 120 ./tools/hbm_calib > "$OUT/bytes.jsonl"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- ./tools/hbm_calib > /dev/null
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- ./tools/hbm_calib > /dev/null
python3 tools/hbm_calib.py "$OUT" | tee "$OUT/summary.json"
