# Proof runs of tools/divsqrt_exhaustive.hip on the GPU box (built there), logs in gpurun_out/dsx
set -e -o pipefail
mkdir -p gpurun_out/dsx
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -Wno-unused-value tools/divsqrt_exhaustive.hip -o /tmp/dsx
for m in "$@"; do
  tag=$(echo "$m" | tr ' ' '_')
  echo "[dsx] $m"
  timeout -k 10 400 /tmp/dsx $m > gpurun_out/dsx/$tag.log 2>&1 || { echo "rc=$? for $m"; tail -3 gpurun_out/dsx/$tag.log; exit 1; }
  tail -1 gpurun_out/dsx/$tag.log
done
