#!/bin/bash
# A/B timing of frame-kernel variants on the 70k-face stand-in (C3 at 1920x1080, and 3840x2160).
# usage: bash scripts/ab_mesh.sh variant...
mkdir -p gpurun_out /tmp/m
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o /tmp/m/s70k.obj > /dev/null || exit 1
export ERAY_AB_MESH=/tmp/m/s70k.obj
timeout -k 10 300 python scripts/ab_variants.py run "$@" > gpurun_out/ab_c3.log 2>&1 || exit 1
if [ "${AB_4K:-0}" = 1 ]; then
  ERAY_AB_W=3840 ERAY_AB_H=2160 timeout -k 10 300 python scripts/ab_variants.py run "$@" > gpurun_out/ab_ns.log 2>&1
fi
