#!/bin/bash
# A/B of environment settings (same library), interleaved: tools/ab_env.sh "VAR=a VAR=b" ROUNDS [perf_probe args...]
# "-" stands for no setting.
SETS=$1; ROUNDS=$2; shift 2
for r in $(seq 1 $ROUNDS); do
  for v in $SETS; do
    echo "== $v round $r"
    if [ "$v" = "-" ]; then timeout -k 10 150 python3 tools/perf_probe.py "$@" || exit 1
    else env "$v" timeout -k 10 150 python3 tools/perf_probe.py "$@" || exit 1; fi
  done
done
