#!/bin/bash
# Build an A/B variant library with one csrc file recompiled under extra
# flags (e.g. -DADAM_U=2).  Usage:
#   tools/build_variant.sh NAME FILE.hip [extra hipcc flags]
# -> abvar/lib_NAME.so (select at run time with IKEA_REC_HIP_LIB=...)
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
obj=ikea-recommender-system_amd/build/obj
base=$(basename "$src" .hip)
mkdir -p abvar
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-result "$@" \
  -I ikea-recommender-system_amd/csrc -c "ikea-recommender-system_amd/csrc/$base.hip" -o abvar/${base}_$name.o
others=$(ls $obj/*.o | grep -v "/$base.o\$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC abvar/${base}_$name.o $others -L/opt/rocm/lib -lrccl -o abvar/lib_$name.so
rm -f abvar/${base}_$name.o
echo abvar/lib_$name.so
