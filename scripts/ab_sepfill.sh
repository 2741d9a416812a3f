#!/bin/bash
# A/B of the separate fill kernel beside the dense detail build (3840x2160 / 70k, C5):
# usage: bash scripts/ab_sepfill.sh "sep dpc fpc" ...
mkdir -p gpurun_out /tmp/m
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o /tmp/m/s70k.obj > /dev/null || exit 1
if [ "${AB_C5:-0}" = 1 ]; then
  python -m eray_amd.meshgen --triangles 1000000 --seed 1234 -o /tmp/m/s1m.obj > /dev/null || exit 1
fi
for cfg in "$@"; do
  set -- $cfg
  echo "separate=$1 detail/CU=$2 fill/CU=$3"
  export ERAY_SEPARATE_FILL=$1 ERAY_SEP_DETAIL_PER_CU=$2 ERAY_SEP_FILL_PER_CU=$3
  ERAY_AB_MESH=/tmp/m/s70k.obj ERAY_AB_W=3840 ERAY_AB_H=2160 timeout -k 10 120 python scripts/ab_variants.py run cur || exit 1
  if [ "${AB_C5:-0}" = 1 ]; then
    ERAY_AB_MESH=/tmp/m/s1m.obj ERAY_AB_W=7680 ERAY_AB_H=4320 timeout -k 10 300 python scripts/ab_variants.py run cur || exit 1
  fi
done
