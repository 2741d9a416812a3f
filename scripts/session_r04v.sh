#!/bin/bash
# Round 4: per-workgroup frame timelines (trace build) of the north-star frame and C2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04v}
mkdir -p $OUT /tmp/eray_meshes
export TMPDIR=/tmp
M=/tmp/eray_meshes
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o $M/standin70k.obj > /dev/null || exit 1
for c in "$M/standin70k.obj 3840 2160" "objects/cube.obj 1920 1080"; do
  echo "=== $c"
  ERAY_LIB=eray_amd/lib/liberay_hip_trace.so timeout -k 10 120 python scripts/wg_trace.py $c 2>&1 | grep -v amdgpu.ids || exit 1
done | tee $OUT/wg_trace.txt
