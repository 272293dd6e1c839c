set -e
O=gpurun_out/r03zw
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
for c in 2 4d 3; do
for f in 64 128 96; do
  timeout -k 10 200 python3 bench.py --config $c --frames-per-launch $f --no-cpu-baseline --reference-loops 0 --no-dedup-check --steps 3 > $O/b_${c}_${f}_$r.json 2> $O/b_${c}_${f}_$r.log
  python3 -c "import json; d=json.load(open('$O/b_${c}_${f}_$r.json')); print('$r $c $f', d['value'], d['ms_per_step'])"
done; done; done
