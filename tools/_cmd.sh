set -e
O=gpurun_out/r03zp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_render_ahead.py -x -q --timeout 200 --timeout-method thread > $O/test_ra.log 2>&1 || { tail -40 $O/test_ra.log; exit 1; }
tail -1 $O/test_ra.log
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.log
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['value_reference_loop'], d['reference_loop'])"
timeout -k 10 300 python3 bench.py --config 4d > $O/bench_4d.json 2> $O/bench_4d.log
python3 -c "import json; d=json.load(open('$O/bench_4d.json')); print(d['value'], d['value_reference_loop'], d['reference_loop'])"
