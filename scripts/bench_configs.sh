#!/bin/bash
# One-GPU bench lines for the BASELINE.json configs (meshes generated on the box), each followed by
# a rocprofv3 kernel-stats run and (PMC=1) the counter passes of the same command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/configs}
mkdir -p $OUT /tmp/eray_meshes
export TMPDIR=/tmp
M=/tmp/eray_meshes
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o $M/standin70k.obj > /dev/null || exit 1
if [ "${WITH_1M:-0}" = 1 ]; then
  python -m eray_amd.meshgen --triangles 1000000 --seed 1234 -o $M/synth1m.obj > /dev/null || exit 1
fi
run() {  # name timeout args...   (ONLY="c2 c3 ...": those configs alone)
  local name=$1 t=$2; shift 2
  if [ -n "${ONLY:-}" ] && [[ " $ONLY " != *" $name "* ]]; then return 0; fi
  echo "=== $name: $*"
  timeout -k 10 "$t" python bench.py "$@" > $OUT/$name.json.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu $OUT/$name.json.log | tail -1 | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
  grep '^{' $OUT/$name.json.log | tail -1 > $OUT/$name.json
  if [ "${PROF:-1}" = 1 ]; then
    timeout -k 10 "$t" rocprofv3 --kernel-trace --stats -d $OUT/prof_$name -o run --output-format csv -- \
        python bench.py "$@" --no-moving-camera --no-cpu-baseline > $OUT/prof_$name.log 2>&1 || exit $?
  fi
  if [ "${PMC:-0}" = 1 ]; then
    PMC_DIR=${OUT#gpurun_out/}/pmc_$name BENCH_ARGS="$* --no-moving-camera --no-cpu-baseline" bash scripts/gpu_pmc.sh || exit $?
  fi
}
run c2 180 --steps 200 ${C2_ARGS:-}
run c3 180 --mesh $M/standin70k.obj --steps 100 --no-cpu-baseline
run ns_4k_70k 240 --mesh $M/standin70k.obj --width 3840 --height 2160 --steps 100 --no-cpu-baseline
run c4_1gpu 120 --width 3840 --height 2160 --steps 100 --no-cpu-baseline
if [ "${WITH_1M:-0}" = 1 ]; then
  run c5_1gpu 400 --mesh $M/synth1m.obj --width 7680 --height 4320 --steps 10 --warmup 3 --no-cpu-baseline
fi
