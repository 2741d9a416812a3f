#!/bin/bash
# Round-3 session d: per-wave binned search — parity on the binned paths, A/B vs the shared
# search (ERAY_RENDER_SHARED_DETAIL), the per-workgroup trace at 3840x2160 / 70k.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out /tmp/eray_meshes
export TMPDIR=/tmp
M=/tmp/eray_meshes
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o $M/standin70k.obj > /dev/null || exit 1
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-12}
  echo "=== $name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  return 0
}
step pytest_binned 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_camera_path.py tests/test_gpu_ring.py tests/test_gpu_render.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider
TAILN=2 step ab_4k70k 200 python scripts/ab_flags.py $M/standin70k.obj 3840 2160 0 32
TAILN=2 step ab_c3 200 python scripts/ab_flags.py $M/standin70k.obj 1920 1080 0 32
TAILN=40 step trace_4k70k 120 env ERAY_LIB=eray_amd/lib/liberay_hip_trace.so python scripts/wg_trace.py $M/standin70k.obj 3840 2160
