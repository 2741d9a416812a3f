#!/bin/bash
# A/B of the working tree (cur) against the last commit (head), twice, on C2, C3, 3840x2160 / 70k
# and the cube at 3840x2160.
mkdir -p gpurun_out /tmp/m
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o /tmp/m/s70k.obj > /dev/null || exit 1
V=${AB_VARIANTS:-"head cur head cur"}
timeout -k 10 120 python scripts/ab_variants.py run $V || exit 1
ERAY_AB_MESH=/tmp/m/s70k.obj timeout -k 10 120 python scripts/ab_variants.py run $V || exit 1
ERAY_AB_MESH=/tmp/m/s70k.obj ERAY_AB_W=3840 ERAY_AB_H=2160 timeout -k 10 120 python scripts/ab_variants.py run $V || exit 1
if [ "${AB_CUBE4K:-1}" = 1 ]; then
  ERAY_AB_W=3840 ERAY_AB_H=2160 timeout -k 10 120 python scripts/ab_variants.py run $V || exit 1
fi
if [ "${AB_C5:-0}" = 1 ]; then
  python -m eray_amd.meshgen --triangles 1000000 --seed 1234 -o /tmp/m/s1m.obj > /dev/null || exit 1
  ERAY_AB_MESH=/tmp/m/s1m.obj ERAY_AB_W=7680 ERAY_AB_H=4320 timeout -k 10 300 python scripts/ab_variants.py run $V || exit 1
fi
