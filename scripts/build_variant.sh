#!/bin/bash
# Diagnostics: a same-source variant of the product library for a same-box A/B.
#   scripts/build_variant.sh NAME SOURCE 'SED-EXPRESSION' ['SED-EXPRESSION' ...]
#   scripts/build_variant.sh NAME SOURCE --from FILE   (FILE replaces eray_amd/csrc/SOURCE)
# compiles eray_amd/csrc/SOURCE with the sed edits applied (into eray_amd/_obj/variant_NAME.o) and
# links it with the product's other objects -> eray_amd/lib/liberay_hip_NAME.so.  Fails when an
# edit matches nothing (the variant would silently equal the product).
set -eu
cd "$(dirname "$0")/.."
NAME=$1; SRC=$2; shift 2
python -m eray_amd.build > /dev/null
O=eray_amd/_obj
TMP=eray_amd/csrc/_variant_$NAME.${SRC##*.}
trap 'rm -f $TMP' EXIT
if [ "${1:-}" = --from ]; then cp "$2" $TMP; shift 2; else cp eray_amd/csrc/$SRC $TMP; fi
for e in "$@"; do
  before=$(md5sum < $TMP)
  sed -i "$e" $TMP
  [ "$before" != "$(md5sum < $TMP)" ] || { echo "edit matched nothing: $e" >&2; exit 1; }
done
F="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function --offload-arch=gfx950 -Iinclude -Ieray_amd/csrc -mllvm -amdgpu-kernarg-preload-count=15"
case $SRC in *.cpp) LANG="-x hip";; *) LANG="";; esac
hipcc $F $LANG -c $TMP -o $O/variant_$NAME.o
objs=""
for s in render.hip setup.hip trace.hip bins.hip shaderlib.hip capi.cpp comm.cpp objload.cpp; do
  [ $s = $SRC ] && objs="$objs $O/variant_$NAME.o" || objs="$objs $O/$s.o"
done
hipcc --offload-arch=gfx950 -shared -fPIC -o eray_amd/lib/liberay_hip_$NAME.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo eray_amd/lib/liberay_hip_$NAME.so
