set -e
O=gpurun_out/r04c
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PTAMD_LIB=optixpathtracer_amd/_variants/lib_grp4.so
echo "[r04c] PMC of the group traversal (SQ, TCC, TCP passes)"
timeout -k 10 500 tools/pmc.sh $O/pmc_grp4 --fpl 64 --spp 64 --modes 1 > $O/pmc_grp4.log 2>&1
tail -1 $O/pmc_grp4.log
echo "[r04c] PMC of the group traversal (TA / TD passes)"
timeout -k 10 400 tools/pmc_ta.sh $O/pmcta_grp4 --fpl 64 --spp 64 --modes 1 > $O/pmcta_grp4.log 2>&1
tail -1 $O/pmcta_grp4.log
python3 tools/pmc_summary.py $O/pmc_grp4 k_trace_pair > $O/pmc_grp4_summary.txt 2>&1 || true
python3 tools/pmc_summary.py $O/pmcta_grp4 k_trace_pair > $O/pmcta_grp4_summary.txt 2>&1 || true
cat $O/pmc_grp4_summary.txt $O/pmcta_grp4_summary.txt
