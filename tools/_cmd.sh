set -e
mkdir -p gpurun_out/r03ze
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 bench.py > gpurun_out/r03ze/bench_default.json 2> gpurun_out/r03ze/bench_default.log
cat gpurun_out/r03ze/bench_default.json
