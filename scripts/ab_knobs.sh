#!/bin/bash
# A/B of the frame kernel's launch knobs (fill share, fill-first role order) on one library:
# C2, C3 and 3840x2160 / 70k.  usage: bash scripts/ab_knobs.sh "share first" ... ("auto -": the launcher's own choice)
mkdir -p gpurun_out /tmp/m
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o /tmp/m/s70k.obj > /dev/null || exit 1
for cfg in "$@"; do
  set -- $cfg
  echo "share=$1 fill_first=$2"
  if [ "$1" = auto ]; then unset ERAY_FILL_SHARE ERAY_FILL_FIRST; else export ERAY_FILL_SHARE=$1 ERAY_FILL_FIRST=$2; fi
  timeout -k 10 120 python scripts/ab_variants.py run cur || exit 1
  ERAY_AB_MESH=/tmp/m/s70k.obj timeout -k 10 120 python scripts/ab_variants.py run cur || exit 1
  ERAY_AB_MESH=/tmp/m/s70k.obj ERAY_AB_W=3840 ERAY_AB_H=2160 timeout -k 10 120 python scripts/ab_variants.py run cur || exit 1
  ERAY_AB_W=3840 ERAY_AB_H=2160 timeout -k 10 120 python scripts/ab_variants.py run cur || exit 1
done
