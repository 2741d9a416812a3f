#!/bin/bash
# A/B: large-mesh frame kernel at 2 vs 3 waves per SIMD, by fill share (C3 and 3840x2160 / 70k).
mkdir -p gpurun_out /tmp/m
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o /tmp/m/s70k.obj > /dev/null || exit 1
export ERAY_AB_MESH=/tmp/m/s70k.obj
for s in 2 3 4; do
  echo "share=$s"
  ERAY_FILL_SHARE=$s timeout -k 10 120 python scripts/ab_variants.py run base occ3 || exit 1
  ERAY_FILL_SHARE=$s ERAY_AB_W=3840 ERAY_AB_H=2160 timeout -k 10 120 python scripts/ab_variants.py run base occ3 || exit 1
done
