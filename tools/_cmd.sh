set -e
O=gpurun_out/r03zt
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for a in "128 64" "128 32" "128 22" "128 16" "256 64" "256 43" "256 32" "512 64" "1024 64"; do
  set -- $a
  timeout -k 10 200 python3 bench.py --spp $1 --frames-per-launch $2 --no-cpu-baseline --reference-loops 0 --no-dedup-check --steps 5 > $O/b_$1_$2.json 2> $O/b_$1_$2.log
  python3 -c "import json; d=json.load(open('$O/b_$1_$2.json')); print('$1 $2', d['value'], d['ms_per_step'])"
done
