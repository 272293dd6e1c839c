set -e
O=gpurun_out/r03h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tools/ab.sh "r16 r12 r20 t16 t24" 4 --fpl 64 --spp 256 --modes 1,3 --repeat 1 > $O/ab.log 2>&1
echo done
