#!/bin/bash
# rocprofv3 kernel-trace stats of tools/perf_probe.py for one scene (repo root, GPU box):
#   tools/kstats.sh OUTDIR SCENE [perf_probe args...]
OUT=$1; SCENE=$2; shift 2
ROOT="$GRAFT_REPO_ROOT"; [ -z "$ROOT" ] && ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && mkdir -p "$OUT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 tools/perf_probe.py --scene "$SCENE" --repeat 1 "$@" > "$OUT/probe.log" 2>&1 || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f'{float(r["TotalDurationNs"])/tot*100:6.1f}%  calls={r["Calls"]:>6}  avg_us={float(r["AverageNs"])/1e3:9.1f}  {r["Name"][:110]}')
PY
