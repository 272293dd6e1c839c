#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=r05zu
for v in m0 m2k m0 m2k; do
  PTAMD_LIB=optixpathtracer_amd/_variants/lib_$v.so timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --reference-loops 512 > gpurun_out/${T}_$v.json 2> gpurun_out/${T}_$v.log || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/${T}_$v.json'));rl=d['reference_loop'];print('$v', d['value'], d['value_reference_loop'], rl['first_call_after_change_ms'], rl['no_render_ahead'])"
done
