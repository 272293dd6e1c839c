#!/bin/bash
# Round evidence on the GPU box (repo root): GPU tests, bench.py on every BASELINE config, and
# tools/profile.sh (rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes) on the headline.
#   tools/round.sh TAG
# Every step has its own time limit and the chain stops at the first failure.
set -e
TAG=${1:-r02}
OUT=gpurun_out/round_$TAG
mkdir -p "$OUT"
echo "[round] gpu tests"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gputest.log" 2>&1
tail -1 "$OUT/gputest.log"
for c in 2 3 4l 5 4d; do
  echo "[round] bench config $c"
  timeout -k 10 300 python3 bench.py --config $c > "$OUT/bench_config$c.json" 2> "$OUT/bench_config$c.log"
  cat "$OUT/bench_config$c.json"
done
echo "[round] profile"
timeout -k 10 900 tools/profile.sh $TAG > "$OUT/profile.log" 2>&1
tail -3 "$OUT/profile.log"
