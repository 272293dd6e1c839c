#!/bin/bash
# Per-kernel rocprofv3 stats of libptamd.so variants (tools/build_variants.sh), one
# perf_probe run each:  tools/ab_kstats.sh "v1 v2" [perf_probe args...]
VARS=$1; shift
ROOT="$GRAFT_REPO_ROOT"; [ -z "$ROOT" ] && ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
for v in $VARS; do
  OUT="$ROOT/gpurun_out/abk_$v"
  PTAMD_LIB=optixpathtracer_amd/_variants/lib_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
    --output-format csv -d "$OUT" -o run -- python3 tools/perf_probe.py --repeat 1 "$@" > "$OUT.log" 2>&1 || exit 1
  echo "== $v"; grep msamples "$OUT.log"
  f=$(find "$OUT" -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print(f'{r["Name"][:90]:90s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:10.1f} us {float(r["Percentage"]):6.2f} %')
PY
done
