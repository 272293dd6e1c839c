set -e
O=gpurun_out/r04p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04p] full GPU suite with the SAH builder as default"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
echo "[r04p] SAH bins 16 / 64 / 256"
tools/ab.sh "bins16 base bins256" 2 --modes 1,3 --fpl 64 --spp 64 --stats > $O/ab_bins.log 2>&1
tools/ab.sh "bins16 base bins256" 1 --scene sponza_class --fpl 64 --spp 64 --stats > $O/ab_bins_sponza.log 2>&1
python3 tools/ab_summary.py $O/ab_bins.log $O/ab_bins_sponza.log
grep -h '"bvh_ms"\|nodes_per_ray' $O/ab_bins.log $O/ab_bins_sponza.log | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l)
    print({k: j[k] for k in ('scene', 'bvh_ms', 'bvh_nodes', 'bvh_depth', 'mode', 'msamples_s', 'nodes_per_ray', 'tris_per_ray') if k in j})"
