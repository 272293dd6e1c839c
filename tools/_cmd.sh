set -e
O=gpurun_out/r03zl
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -2 $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.log
cat $O/bench_default.json
