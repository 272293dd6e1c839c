set -e
O=gpurun_out/r03l
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PTAMD_LIB=optixpathtracer_amd/_variants/lib_pad.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bitexact.py tests/test_gpu_determinism.py -x -q --timeout 200 --timeout-method thread > $O/test_pad.log 2>&1
tail -1 $O/test_pad.log
for v in nb pad; do
  PTAMD_LIB=optixpathtracer_amd/_variants/lib_$v.so timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES --output-format csv -d $O/pmc_$v -o run -- python3 tools/perf_probe.py --spp 64 --fpl 64 --modes 1 --repeat 1 > $O/pmc_$v.log 2>&1
  python3 tools/pmc_summary.py $O/pmc_$v k_trace_pair > $O/pmc_$v.txt
  echo "== $v"; cat $O/pmc_$v.txt
done
tools/ab.sh "nb ne pad base" 3 --fpl 64 --spp 256 --modes 1,3,2 --repeat 1 > $O/ab.log 2>&1
python3 tools/ab_summary.py $O/ab.log
