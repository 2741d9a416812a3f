#!/bin/bash
# Diagnostics library: the product objects with render.hip replaced by the per-workgroup
# timestamp build (scripts/microbench/render_trace.hip) -> eray_amd/lib/liberay_hip_trace.so.
set -eu
cd "$(dirname "$0")/.."
python -m eray_amd.build > /dev/null
O=eray_amd/_obj
F="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function --offload-arch=gfx950 -Iinclude -Ieray_amd/csrc -mllvm -amdgpu-kernarg-preload-count=15"
hipcc $F -c scripts/microbench/render_trace.hip -o $O/render_trace.o
objs=""
for s in setup.hip trace.hip bins.hip shaderlib.hip capi.cpp comm.cpp objload.cpp; do objs="$objs $O/$s.o"; done
hipcc --offload-arch=gfx950 -shared -fPIC -o eray_amd/lib/liberay_hip_trace.so $O/render_trace.o $objs \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo eray_amd/lib/liberay_hip_trace.so
