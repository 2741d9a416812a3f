#!/bin/bash
# rocprofv3 kernel stats of the larger BASELINE configs on one GPU (C3, the north-star
# 3840x2160 / 70k frame, C5's frame); summaries land in gpurun_out/prof_<name>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out /tmp/eray_meshes
export TMPDIR=/tmp
M=/tmp/eray_meshes
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o $M/standin70k.obj > /dev/null || exit 1
python -m eray_amd.meshgen --triangles 1000000 --seed 1234 -o $M/synth1m.obj > /dev/null || exit 1
prof() {  # name timeout bench-args...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run --output-format csv -- \
      python bench.py --no-cpu-baseline "$@" > gpurun_out/prof_$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 gpurun_out/prof_$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
prof c3 240 --mesh $M/standin70k.obj --steps 100
prof ns_4k_70k 240 --mesh $M/standin70k.obj --width 3840 --height 2160 --steps 100
prof c5 400 --mesh $M/synth1m.obj --width 7680 --height 4320 --scaling strong --steps 10
