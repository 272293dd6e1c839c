set -e
O=gpurun_out/r04g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04g] band-split GPU tests + parity subset"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_band_split.py tests/test_gpu_render_ahead.py tests/test_gpu_bitexact.py \
  tests/test_gpu_debug_path.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1 \
  || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
echo "[r04g] one-frame path"
for s in sphere_box_diffuse sphere_box_dielectric20 sphere_box_conductor; do
  timeout -k 10 200 python3 tools/one_frame.py --scene $s
done > $O/one_frame.log 2>&1
cat $O/one_frame.log | grep scene
