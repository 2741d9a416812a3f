#!/bin/bash
# Round-3 session: GPU tests, frames-in-flight sweep, bench (N=1) and the N=2 plumbing rehearsal.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out /tmp/eray_meshes
export TMPDIR=/tmp
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o /tmp/eray_meshes/standin70k.obj > /dev/null || exit 1
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
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step fif 400 python -u scripts/frames_in_flight.py --big
TAILN=100 step fill_mlp 200 scripts/microbench/fill_mlp
TAILN=1 step bench 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 3
TAILN=1 step bench20 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
TAILN=1 step rehearsal_n2 300 env ERAY_BENCH_REHEARSAL=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 40 --warmup 5
