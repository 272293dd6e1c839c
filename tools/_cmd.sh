set -e
O=gpurun_out/r04j
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04j] band tests"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_band_split.py tests/test_gpu_render_ahead.py tests/test_gpu_parity.py -x -q \
  --timeout 200 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
echo "[r04j] one-frame path: 7/16 + 9/16 bands, first band downloaded early"
for r in 1 2; do for s in sphere_box_diffuse sphere_box_dielectric20 sphere_box_conductor; do
  timeout -k 10 200 python3 tools/one_frame.py --scene $s --repeat 3
done; done > $O/one_frame.log 2>&1
grep scene $O/one_frame.log | cut -c1-170
echo "[r04j] trace workgroup size A/B (256 / 512 / 768 threads, 49 / 100 / 150 staged nodes)"
tools/ab.sh "base tb512 tb768" 3 --modes 1,3,2,0 --fpl 64 --spp 64 > $O/ab_trace_block.log 2>&1
tools/ab.sh "base tb512 tb768" 2 --scene sponza_class --fpl 64 --spp 64 > $O/ab_trace_block_sponza.log 2>&1
python3 tools/ab_summary.py $O/ab_trace_block.log $O/ab_trace_block_sponza.log
