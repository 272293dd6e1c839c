set -e
O=gpurun_out/r04u
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1 \
  || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
