set -e
O=gpurun_out/r03zu
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SECONDS=0; timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log; echo "smoke $SECONDS s"; SECONDS=0
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.log
echo "bench $SECONDS s"
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['value_reference_loop'], d['mse_vs_oracle']['mse'])"
