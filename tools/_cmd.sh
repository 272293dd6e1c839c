#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=r05zk
timeout -k 10 600 tools/ab.sh "base" 3 --scene sphere_box_diffuse --fpl 64 --spp 128 --modes 1,2 --streams 1,2 > gpurun_out/${T}_streams.log 2>&1 || exit 1
timeout -k 10 400 tools/ab.sh "base" 2 --scene sponza_class --fpl 64 --spp 64 --streams 1,2 > gpurun_out/${T}_streams_c5.log 2>&1 || exit 1
timeout -k 10 400 tools/ab.sh "base" 2 --scene sphere_box_dielectric20 --fpl 64 --spp 128 --streams 1,2 > gpurun_out/${T}_streams_4d.log 2>&1 || exit 1
grep -h '"msamples_s"' gpurun_out/${T}_streams*.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['mode'], d.get('streams'), d['msamples_s'])"
