#!/bin/bash
# Round evidence on the GPU box (repo root), in two gpurun calls (each under gpurun's limit),
# profile FIRST, so the bench lines read PMC figures of their own sources:
#   tools/round.sh TAG profile  tools/profile.sh (rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE
#                               passes) on the headline, the SQ/TCC/TCP passes of tools/pmc.sh
#                               for profiles/valu.json, the TA/TD passes of tools/pmc_ta.sh for
#                               profiles/vmem.json, the k_shade_nee VALU passes and kernel stats of
#                               configs 3 and 5; then, here: tools/store_round.py TAG profile
#   tools/round.sh TAG bench    GPU tests, then bench.py on every BASELINE config; then, here:
#                               tools/store_round.py TAG bench
# Every step has its own time limit and the chain stops at the first failure.
set -e
TAG=${1:-r03}
PART=${2:-bench}
OUT=gpurun_out/round_$TAG
mkdir -p "$OUT"
if [ "$PART" = bench ]; then
  echo "[round] gpu tests"
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gputest.log" 2>&1
  tail -1 "$OUT/gputest.log"
  for c in 2 3 4l 5 5t 4d; do
    echo "[round] bench config $c"
    timeout -k 10 300 python3 bench.py --config $c > "$OUT/bench_config$c.json" 2> "$OUT/bench_config$c.log"
    cat "$OUT/bench_config$c.json"
  done
else
  echo "[round] profile"
  timeout -k 10 900 tools/profile.sh $TAG > "$OUT/profile.log" 2>&1
  tail -3 "$OUT/profile.log"
  echo "[round] pmc (SQ / TCC / TCP passes, Lambert, 128 frames)"
  timeout -k 10 600 tools/pmc.sh gpurun_out/pmc_$TAG --fpl 128 --spp 128 > "$OUT/pmc.log" 2>&1
  tail -1 "$OUT/pmc.log"
  echo "[round] pmc (TA / TD / TCP passes, Lambert, 128 frames)"
  timeout -k 10 600 tools/pmc_ta.sh gpurun_out/pmcta_$TAG --fpl 128 --spp 128 > "$OUT/pmc_ta.log" 2>&1
  tail -1 "$OUT/pmc_ta.log"
  # VALU issue of k_shade_nee, the dominant kernel of the Default / Layered configs (bench.py
  # roofline.valu reads profiles/shade_valu_config<C>.json): one SQ pass per config
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  for c in 3:sphere_box_conductor 4l:sphere_box_layered 5:sponza_class; do
    cfg=${c%%:*}; sc=${c#*:}
    echo "[round] shade VALU pass, config $cfg"
    timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU \
      --output-format csv -d "$OUT/shv_$cfg" -o run -- python3 tools/perf_probe.py --scene $sc --fpl 128 --spp 128 --repeat 1 \
      > "$OUT/shv_$cfg.log" 2>&1
    python3 tools/pmc_summary.py "$OUT/shv_$cfg" k_shade_nee --shade-json "$OUT/shade_valu_config$cfg.json" \
      --source "tools/round.sh $TAG profile (rocprofv3 SQ pass, perf_probe --scene $sc --fpl 128 --spp 128)" | tail -3
  done
  # kernel stats of the Default-mode configs' own bench command
  for cfg in 3 5; do
    echo "[round] kernel trace, config $cfg"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_config$cfg" -o run -- \
      python3 bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline --no-dedup-check --reference-loops 0 \
      > "$OUT/kt_config$cfg.json" 2> "$OUT/kt_config$cfg.log"
    # the same on one wavefront stream: solo kernel times (with two streams a short kernel's
    # window includes the time its workgroups wait behind the other stream's kernels)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt1_config$cfg" -o run -- \
      python3 bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline --no-dedup-check --reference-loops 0 \
      --wavefront-streams 1 > "$OUT/kt1_config$cfg.json" 2> "$OUT/kt1_config$cfg.log"
  done
fi
