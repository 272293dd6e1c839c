set -o pipefail
mkdir -p gpurun_out/r06kt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in 5t 4l; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06kt/kt1_config$cfg -o run -- \
    python3 bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline --no-dedup-check --reference-loops 0 \
    --wavefront-streams 1 > gpurun_out/r06kt/kt1_config$cfg.json 2> gpurun_out/r06kt/kt1_config$cfg.log || exit 1
  echo "config $cfg done"
done
