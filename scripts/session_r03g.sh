#!/bin/bash
# Round-3 session g: dynamic detail scheduling — binned parity tests, A/B vs static rounds.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out /tmp/eray_meshes
export TMPDIR=/tmp
M=/tmp/eray_meshes
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o $M/standin70k.obj > /dev/null || exit 1
: > gpurun_out/ab_snake.log
for rep in 1 2; do
  for v in base ff s225 ffs17; do
    if [ $v = base ]; then L=eray_amd/lib/liberay_hip.so; else L=eray_amd/lib/liberay_hip_$v.so; fi
    for cfg in "3840 2160" "1920 1080"; do
      out=$(ERAY_LIB=$L timeout -k 10 120 python scripts/ab_flags.py $M/standin70k.obj $cfg 0 2>/dev/null | tail -1)
      rc=$?
      echo "$v $cfg $out" | tee -a gpurun_out/ab_snake.log
      if [ $rc -ne 0 ]; then exit $rc; fi
    done
  done
done
