#!/bin/bash
# Round-2 measurement session: GPU tests + smoke, the C2 bench line (CPU baseline), rocprofv3
# kernel stats, PMC traffic for C2, C3, 3840x2160/70k and C5, the other configs' lines, tile
# balance and the one-GPU multi-rank rehearsals.  Every GPU step has its own time limit; a crash,
# abort or time-out ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out /tmp/eray_meshes
export TMPDIR=/tmp
M=/tmp/eray_meshes
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping"; exit $rc; fi
  return 0
}
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o $M/standin70k.obj > /dev/null || exit 1
python -m eray_amd.meshgen --triangles 1000000 --seed 1234 -o $M/synth1m.obj > /dev/null || exit 1
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 600 python bench.py --steps 200 --warmup 20 --cpu-seconds 10
step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline
for cfg in "c2|--steps 50 --warmup 5" "c3|--mesh $M/standin70k.obj --steps 50 --warmup 5" \
           "ns_4k_70k|--mesh $M/standin70k.obj --width 3840 --height 2160 --steps 30 --warmup 5" \
           "c5_1gpu|--mesh $M/synth1m.obj --width 7680 --height 4320 --scaling strong --steps 5 --warmup 2"; do
  name=${cfg%%|*}; args=${cfg#*|}
  PMC_DIR=pmc_$name BENCH_ARGS="$args --no-cpu-baseline --no-moving-camera" bash scripts/gpu_pmc.sh > gpurun_out/pmc_$name.out 2>&1
  rc=$?; echo "=== pmc $name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_$name.out; exit $rc; fi
done
step cfg_c3 300 python bench.py --no-cpu-baseline --mesh $M/standin70k.obj --steps 100
step cfg_ns_4k_70k 300 python bench.py --no-cpu-baseline --mesh $M/standin70k.obj --width 3840 --height 2160 --steps 50
step cfg_c4_1gpu 300 python bench.py --no-cpu-baseline --width 3840 --height 2160 --scaling strong --steps 100
step cfg_c5_1gpu 400 python bench.py --no-cpu-baseline --mesh $M/synth1m.obj --width 7680 --height 4320 --scaling strong --steps 5
for n in 2 4; do
  step rehearsal_n$n 300 env ERAY_BENCH_REHEARSAL=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 50 --warmup 5
done
