set -e
V=optixpathtracer_amd/_variants
for sc in sphere_box_layered sphere_box_conductor sponza_class; do
  for k in 1 0; do
    PTAMD_LIB=$V/lib_nofuse.so timeout -k 10 120 python3 tools/render_npy.py gpurun_out/a_$sc$k.npy --scene $sc --kernel $k
    PTAMD_LIB=$V/lib_reuse.so timeout -k 10 120 python3 tools/render_npy.py gpurun_out/b_$sc$k.npy --scene $sc --kernel $k
    python3 tools/render_npy.py --compare gpurun_out/a_$sc$k.npy gpurun_out/b_$sc$k.npy
  done
done
tools/ab.sh "fuse reuse" 2 --fpl 16 --spp 32 --modes 0,4 --scene sphere_box_conductor
