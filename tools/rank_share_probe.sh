#!/bin/bash
# One rank's share of a strong-scaling step, measured on one GPU: under
# strong scaling an N-GPU step gives each rank spp/N frames, so the 1 -> N projection is the rate
# of bench.py at --spp spp/N against --spp spp.  Run from the repo root on the GPU box:
#   tools/rank_share_probe.sh OUTDIR
set -e
OUT=${1:-gpurun_out/rank_share}
mkdir -p "$OUT"
run() {  # config spp steps
  timeout -k 10 300 python3 bench.py --config $1 --spp $2 --steps $3 --warmup 1 --no-cpu-baseline --no-dedup-check \
    --reference-loops 0 > "$OUT/c$1_spp$2.json" 2> "$OUT/c$1_spp$2.log"
  python3 -c "import json,sys; d=json.load(open('$OUT/c$1_spp$2.json')); print('$1', $2, d['value'], d['ms_per_step'], d['config']['batch_frames'], d['config']['wavefront_streams'])"
}
for spp in 1024 512 256 128; do run 2 $spp 3; done
for spp in 4096 512; do run 4d $spp 2; done
for spp in 4096 512; do run 4l $spp 2; done
echo rank-share-done
