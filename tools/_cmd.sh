set -e
O=gpurun_out/r04f
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04f] one-frame batches on one and two streams"
timeout -k 10 300 python3 tools/perf_probe.py --fpl 1,2 --streams 1,2 --spp 64 --modes 1,3 > $O/fpl1_streams.log 2>&1
grep msamples $O/fpl1_streams.log | cut -c1-200
