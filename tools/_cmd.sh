set -o pipefail
mkdir -p gpurun_out/r06z2
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06z2/gputest.log 2>&1 || { tail -30 gpurun_out/r06z2/gputest.log; exit 1; }
tail -1 gpurun_out/r06z2/gputest.log
