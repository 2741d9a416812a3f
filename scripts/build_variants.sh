#!/bin/bash
# Diagnostics: product libraries with render.hip (or VARIANT_SRC) compiled under other compile-time
# choices, for same-box A/B runs (ERAY_LIB selects one).  Usage: build_variants.sh name "-DMACRO=value ..." ...
set -eu
cd "$(dirname "$0")/.."
python -m eray_amd.build > /dev/null
O=eray_amd/_obj
F="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function --offload-arch=gfx950 -Iinclude -mllvm -amdgpu-kernarg-preload-count=15"
V=${VARIANT_SRC:-render.hip}
objs=""
for s in render.hip setup.hip trace.hip bins.hip shaderlib.hip capi.cpp comm.cpp objload.cpp; do
  [ "$s" = "$V" ] || objs="$objs $O/$s.o"
done
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  lang=""; case $V in *.cpp) lang="-x hip";; esac
  hipcc $F $defs $lang -c eray_amd/csrc/$V -o $O/variant_$name.o
  hipcc --offload-arch=gfx950 -shared -fPIC -o eray_amd/lib/liberay_hip_$name.so $O/variant_$name.o $objs \
      -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo eray_amd/lib/liberay_hip_$name.so
done
