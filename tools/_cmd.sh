set -o pipefail
mkdir -p gpurun_out/r06za
for s in sponza_class:c5 sphere_box_conductor:c3 sphere_box_layered:4l sponza_textured:c5t sphere_box_diffuse:c2; do
  sc=${s%%:*}; tag=${s#*:}
  tools/ab.sh "base ilp" 3 --scene $sc --fpl 128 --spp 256 --repeat 2 > gpurun_out/r06za/ab_ilp_$tag.log 2>&1 || exit 1
done
python3 tools/ab_summary.py gpurun_out/r06za/ab_ilp_*.log
