set -o pipefail
mkdir -p gpurun_out/r06v
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for sc in sphere_box_conductor sponza_class; do
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM \
    --output-format csv -d gpurun_out/r06v/smp_$sc -o run -- python3 tools/perf_probe.py --scene $sc --fpl 128 --spp 128 --repeat 1 > gpurun_out/r06v/smp_$sc.log 2>&1 || exit 1
  for k in k_shade_smp k_shade_nee k_shade_a; do echo "== $sc $k"; python3 tools/pmc_summary.py gpurun_out/r06v/smp_$sc $k --waves 5 | tail -12; done
done
