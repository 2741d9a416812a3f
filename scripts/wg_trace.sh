#!/bin/bash
# Per-workgroup frame timelines (trace build, scripts/build_trace.sh) for the cube at 1920x1080 (one
# frame, and C2's 8 frames per launch into 8 slots), C3, 3840x2160 / 70k in one ring slot and in
# four (beyond the Infinity Cache), and the cube at 3840x2160 ($CASES: a |-separated subset).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out /tmp/eray_meshes
M=/tmp/eray_meshes
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o $M/standin70k.obj > /dev/null || exit 1
export ERAY_LIB=eray_amd/lib/liberay_hip_trace.so
CASES=${CASES:-"objects/cube.obj 1920 1080|objects/cube.obj 1920 1080 8 8|$M/standin70k.obj 1920 1080|$M/standin70k.obj 3840 2160|$M/standin70k.obj 3840 2160 4|objects/cube.obj 3840 2160"}
IFS='|' read -ra LIST <<< "$CASES"
for c in "${LIST[@]}"; do
  echo "=== $c"
  timeout -k 10 120 python scripts/wg_trace.py $c || exit 1
done
