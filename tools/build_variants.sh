#!/bin/bash
# Build A/B variants of the head kernels as whole libraries under variants/
# (pick one at run time with IKEA_REC_HIP_LIB=...).  Usage:
#   tools/build_variants.sh NAME [extra hipcc flags] [--head FILE]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
head=ikea-recommender-system_amd/csrc/head.hip
flags=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--head" ]; then head=$2; shift 2; else flags+=("$1"); shift; fi
done
obj=ikea-recommender-system_amd/build/obj
mkdir -p variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result "${flags[@]}" \
  -I ikea-recommender-system_amd/csrc -c "$head" -o variants/head_$name.o
others=$(ls $obj/*.o | grep -v '/head.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC variants/head_$name.o $others -o variants/lib_$name.so
rm -f variants/head_$name.o
echo variants/lib_$name.so
