set -e
O=gpurun_out/r04h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04h] parity of the hemisphere-split NEE buckets"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bitexact.py tests/test_gpu_parity.py tests/test_gpu_timed_config.py \
  tests/test_gpu_debug_path.py -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
echo "[r04h] A/B"
tools/ab.sh "base nsplit" 3 --scene sphere_box_conductor --fpl 64 --spp 64 > $O/ab_c3.log 2>&1
tools/ab.sh "base nsplit" 2 --scene sphere_box_layered --fpl 64 --spp 64 > $O/ab_4l.log 2>&1
tools/ab.sh "base nsplit" 2 --scene sponza_class --fpl 64 --spp 64 > $O/ab_5.log 2>&1
python3 tools/ab_summary.py $O/ab_c3.log $O/ab_4l.log $O/ab_5.log
