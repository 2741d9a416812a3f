#!/bin/bash
# One-GPU bench lines for the larger BASELINE.json configs (meshes generated on the box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/configs /tmp/eray_meshes
export TMPDIR=/tmp
M=/tmp/eray_meshes
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o $M/standin70k.obj > /dev/null || exit 1
if [ "${WITH_1M:-0}" = 1 ]; then
  python -m eray_amd.meshgen --triangles 1000000 --seed 1234 -o $M/synth1m.obj > /dev/null || exit 1
fi
run() {  # name timeout args...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" python bench.py --no-cpu-baseline "$@" > gpurun_out/configs/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 gpurun_out/configs/$name.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run c2 120 --steps 200
run c3 180 --mesh $M/standin70k.obj --steps 100
run ns_4k_70k 240 --mesh $M/standin70k.obj --width 3840 --height 2160 --steps 50
run c4_1gpu 120 --width 3840 --height 2160 --scaling strong --steps 100
if [ "${WITH_1M:-0}" = 1 ]; then
  run c5_1gpu 400 --mesh $M/synth1m.obj --width 7680 --height 4320 --scaling strong --steps 5
fi
if [ "${REHEARSE:-0}" = 1 ]; then  # the N > 1 path, every rank on GPU 0 (gloo): plumbing only
  for n in 2 4; do
    echo "=== rehearsal n=$n"
    ERAY_BENCH_REHEARSAL=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 50 --warmup 5 \
      > gpurun_out/configs/rehearsal_n$n.log 2>&1 || exit 1
    tail -1 gpurun_out/configs/rehearsal_n$n.log
  done
fi
