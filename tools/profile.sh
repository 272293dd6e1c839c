#!/bin/bash
# Round profile on the GPU box (repo root): bench JSON, rocprofv3 kernel-trace stats of the
# same bench command, PMC traffic passes (FETCH_SIZE / WRITE_SIZE in separate runs, as
# MI355X_MICROARCH.md prescribes) and profiles/traffic.json for bench.py's roofline.traffic.
#   tools/profile.sh TAG [bench args...]
set -e
TAG=${1:-r01}; shift || true
ARGS="$@"
ROOT="$GRAFT_REPO_ROOT"; [ -z "$ROOT" ] && ROOT=$(pwd)
OUT="$ROOT/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT"
echo "[profile] kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-dedup-check --reference-loops 0 $ARGS > "$OUT/kt_bench.json" 2> "$OUT/kt_bench.log"
echo "[profile] kernel trace, one stream (solo kernel times: tools/shade_pmc.py, roofline.single_stream)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt1" -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-dedup-check --reference-loops 0 --wavefront-streams 1 $ARGS > "$OUT/kt1_bench.json" 2> "$OUT/kt1_bench.log"
echo "[profile] FETCH_SIZE"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
  python3 bench.py --steps 1 --warmup 0 --spp 128 --no-cpu-baseline --no-dedup-check --reference-loops 0 $ARGS > "$OUT/fetch.json" 2> "$OUT/fetch.log"
echo "[profile] WRITE_SIZE"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
  python3 bench.py --steps 1 --warmup 0 --spp 128 --no-cpu-baseline --no-dedup-check --reference-loops 0 $ARGS > "$OUT/write.json" 2> "$OUT/write.log"
echo "[profile] read requests by size"
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d "$OUT/rdsz" -o run -- \
  python3 bench.py --steps 1 --warmup 0 --spp 128 --no-cpu-baseline --no-dedup-check --reference-loops 0 $ARGS > "$OUT/rdsz.json" 2> "$OUT/rdsz.log"
python3 tools/traffic.py "$OUT" > "$OUT/traffic.json"
cat "$OUT/traffic.json"
echo "[profile] done"
