#!/bin/bash
# Round-3 session c: per-workgroup traces (4K/70k, C3, C2), the C3 oracle-digest test, bench at
# the new frames-per-launch rule, rocprofv3 kernel stats and PMC passes of the C2 bench.
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
TAILN=40 step trace_4k70k 120 env ERAY_LIB=eray_amd/lib/liberay_hip_trace.so python scripts/wg_trace.py $M/standin70k.obj 3840 2160
TAILN=40 step trace_c3 120 env ERAY_LIB=eray_amd/lib/liberay_hip_trace.so python scripts/wg_trace.py $M/standin70k.obj 1920 1080
TAILN=40 step trace_c2 120 env ERAY_LIB=eray_amd/lib/liberay_hip_trace.so python scripts/wg_trace.py objects/cube.obj 1920 1080
step pytest_c3 300 python -u -m pytest tests/test_gpu_configs.py -q -k c3 --timeout 300 --timeout-method thread -p no:cacheprovider
TAILN=1 step bench 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 10
step rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline
PMC_DIR=pmc_c2 step pmc 600 bash scripts/gpu_pmc.sh
