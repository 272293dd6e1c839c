#!/bin/bash
# Interleaved A/B of the queue budget (pt_set_queue_budget default vs none) on config 4d, the
# two-stream Dielectric config whose batch the default budget lowers to 89 frames.
for r in 1 2 3; do for b in 0 -1; do
timeout -k 10 200 python3 bench.py --config 4d --spp 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-dedup-check --reference-loops 0 --queue-budget $b > gpurun_out/r06h_ab_budget_4d_${r}_${b}.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r06h_ab_budget_4d_${r}_${b}.json')); print('budget $b round $r', d['value'], d['config']['batch_frames'], d['config']['queue_bytes'])"
done; done
