set -e
O=gpurun_out/r03zx
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
for c in 2 4d 3; do
for s in 2 3 4; do
  timeout -k 10 200 python3 bench.py --config $c --wavefront-streams $s --no-cpu-baseline --reference-loops 0 --no-dedup-check --steps 3 > $O/b_${c}_${s}_$r.json 2> $O/b_${c}_${s}_$r.log
  python3 -c "import json; d=json.load(open('$O/b_${c}_${s}_$r.json')); print('$r $c $s', d['value'], d['ms_per_step'])"
done; done; done
