#!/bin/bash
# Round-3 session e: same-box A/B of compile-time variants of the large-mesh detail build
# (candidate batch, workgroups per CU, detail share), 3840x2160 / 70k and C3.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out /tmp/eray_meshes
export TMPDIR=/tmp
M=/tmp/eray_meshes
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o $M/standin70k.obj > /dev/null || exit 1
: > gpurun_out/ab_variants.log
for rep in 1 2; do
  for v in base b4w3 b1w4 b1w4s3 b1w4s4; do
    if [ $v = base ]; then L=eray_amd/lib/liberay_hip.so; else L=eray_amd/lib/liberay_hip_$v.so; fi
    for cfg in "3840 2160" "1920 1080"; do
      out=$(ERAY_LIB=$L timeout -k 10 120 python scripts/ab_flags.py $M/standin70k.obj $cfg 0 2>/dev/null | tail -1)
      rc=$?
      echo "$v $cfg $out" | tee -a gpurun_out/ab_variants.log
      if [ $rc -ne 0 ]; then exit $rc; fi
    done
  done
done
ERAY_LIB=eray_amd/lib/liberay_hip_b1w4s3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -q -x -k "north_star or c3" --timeout 300 --timeout-method thread -p no:cacheprovider 2>&1 | tail -3
