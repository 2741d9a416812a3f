#!/bin/bash
# A/B on one box: C5's moving-camera loop with bin_pairs built for 1 (product), 6 or 8 waves per SIMD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_pairs
mkdir -p $OUT /tmp/eray_meshes
python -m eray_amd.meshgen --triangles 1000000 --seed 1234 -o /tmp/eray_meshes/synth1m.obj > /dev/null || exit 1
for rep in 1 2; do
  for v in "" pw6 pw8; do
    name=${v:-base}$rep
    if [ -n "$v" ]; then export ERAY_LIB=$PWD/eray_amd/lib/liberay_hip_$v.so; else unset ERAY_LIB; fi
    timeout -k 10 200 python scripts/moving_camera.py --mesh /tmp/eray_meshes/synth1m.obj --width 7680 --height 4320 --frames 32 > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }
    echo "$name $(grep moving $OUT/$name.log)"
  done
done
