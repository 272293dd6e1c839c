set -e
O=gpurun_out/r03f
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in split lqsplit; do
PTAMD_LIB=optixpathtracer_amd/_variants/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bitexact.py tests/test_gpu_timed_config.py tests/test_gpu_parity.py tests/test_gpu_debug_path.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/test_$v.log 2>&1
tail -1 $O/test_$v.log
done
tools/ab.sh "base split lqsplit" 3 --fpl 64 --spp 256 --modes 1,3,2 --repeat 1 > $O/ab.log 2>&1
echo done
