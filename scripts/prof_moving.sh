#!/bin/bash
# rocprofv3 kernel statistics of moving-camera frame loops (scripts/moving_camera.py): C2, C3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out /tmp/eray_meshes
export TMPDIR=/tmp
M=/tmp/eray_meshes
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o $M/standin70k.obj > /dev/null || exit 1
prof() {  # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mv_$name -o run --output-format csv -- \
      python scripts/moving_camera.py "$@" > gpurun_out/prof_mv_$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 gpurun_out/prof_mv_$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
prof c2 120
prof c3 180 --mesh $M/standin70k.obj
