#!/bin/bash
# An alternative libsiddhi_hip.so with one source recompiled under extra defines, for tools/ab_lib.sh:
#   tools/build_variant.sh <name> <source.hip> "<-DFOO=1 ...>"  ->  ab/lib_<name>.so
set -e
cd "$(dirname "$0")/../siddhi_amd/csrc"
make -s -j8 >/dev/null
mkdir -p ../../ab/obj
name=$1; src=$2; defs=$3
obj=../../ab/obj/${src%.hip}_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math $defs -c $src -o $obj
objs=$(ls build/*.o | grep -v "build/${src%.hip}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../ab/lib_$name.so $objs $obj -lhiprtc -lrccl
echo ab/lib_$name.so
