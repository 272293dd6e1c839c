set -e
O=gpurun_out/r03zv
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/one_frame_gaps.py > $O/one_frame.json 2> $O/one_frame.log
cat $O/one_frame.json
