set -o pipefail
mkdir -p gpurun_out/r06z8
for s in sphere_box_diffuse:c2 sponza_class:c5 sphere_box_dielectric20:c4d; do
  sc=${s%%:*}; tag=${s#*:}
  tools/ab.sh "full half" 3 --scene $sc --fpl 128 --spp 256 --repeat 2 --stats > gpurun_out/r06z8/ab_half_$tag.log 2>&1 || exit 1
done
python3 tools/ab_summary.py gpurun_out/r06z8/ab_half_*.log
