set -o pipefail
mkdir -p gpurun_out/r06z4
tools/ab.sh "c256 p60 p80 p40 p60b" 4 --scene sphere_box_diffuse --fpl 128 --spp 256 --repeat 2 > gpurun_out/r06z4/ab_pool2_c2.log 2>&1 || exit 1
python3 tools/ab_summary.py gpurun_out/r06z4/ab_pool2_*.log
