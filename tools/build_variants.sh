#!/bin/bash
# Build kernel A/B variants of libptamd.so into optixpathtracer_amd/_variants/ (git-ignored,
# shipped to the GPU box).  Select one at run time with PTAMD_LIB=<path>.
#   tools/build_variants.sh name "-DMACRO=1 ..." [name2 "flags2" ...]
set -e
cd "$(dirname "$0")/../optixpathtracer_amd/csrc"
mkdir -p ../_variants
while [ $# -ge 2 ]; do
  make -s -j8 OUT=../_variants/lib_$1.so OBJDIR=../../build/var_$1 VARIANT="$2"
  shift 2
done
