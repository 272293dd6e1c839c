set -e
O=gpurun_out/r03zh
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PTAMD_LIB=optixpathtracer_amd/_variants/lib_ea.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bitexact.py tests/test_gpu_timed_config.py tests/test_gpu_determinism.py -x -q --timeout 200 --timeout-method thread > $O/test_ea.log 2>&1 || { tail -30 $O/test_ea.log; exit 1; }
tail -1 $O/test_ea.log
tools/ab.sh "base ea" 3 --fpl 64 --spp 256 --modes 1,3,2 --repeat 1 > $O/ab.log 2>&1
python3 tools/ab_summary.py $O/ab.log
