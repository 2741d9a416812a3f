#!/bin/bash
# The frame kernel's two halves alone (x_nofill: detail work only; x_nodetail: fill only) beside
# the full kernel, for C2, C3, 3840x2160 / 70k and the cube at 3840x2160.
mkdir -p gpurun_out /tmp/m
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o /tmp/m/s70k.obj > /dev/null || exit 1
V="cur x_nofill x_nodetail"
timeout -k 10 120 python scripts/ab_variants.py run $V || exit 1
ERAY_AB_MESH=/tmp/m/s70k.obj timeout -k 10 120 python scripts/ab_variants.py run $V || exit 1
ERAY_AB_MESH=/tmp/m/s70k.obj ERAY_AB_W=3840 ERAY_AB_H=2160 timeout -k 10 120 python scripts/ab_variants.py run $V || exit 1
ERAY_AB_W=3840 ERAY_AB_H=2160 timeout -k 10 120 python scripts/ab_variants.py run $V || exit 1
