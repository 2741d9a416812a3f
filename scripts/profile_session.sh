#!/bin/bash
# A round's profiles at the current product (a bench step = one batch of frames): the GPU suite, the driver's bench command, its per-leg
# rocprof rows (ROCTx ranges + kernel trace), and frame-kernel counter passes for C2 and the two
# north_star ring sizes (each counter group its own run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:?set TAG, e.g. r05/final}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAIL\|Error" $OUT/tests.log | head -150; exit $rc; }
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; [ $rc -eq 0 ] || { tail -c 3000 $OUT/bench.err; exit $rc; }
cat $OUT/bench.json | cut -c1-600
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err
rc=$?; [ $rc -eq 0 ] || { tail -c 3000 $OUT/bench_prof.err; exit $rc; }
[ "${NO_PMC:-0}" = 1 ] && exit 0
pass() {  # dir name bench-args counters...
  local d=$1 name=$2 args=$3; shift 3
  mkdir -p $OUT/$d
  timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-include-regex 'frame_kernel|fill_kernel' --output-format csv -d $OUT/$d/$name -o $name -- python3 bench.py $args > $OUT/$d/$name.log 2>&1
  local rc=$?
  echo "pmc $d/$name rc=$rc"
  [ $rc -eq 0 ] || { tail -20 $OUT/$d/$name.log; exit $rc; }
}
C2ARGS="--steps 25 --warmup 3 --no-cpu-baseline --no-moving-camera --no-north-star"
for d in c2:"$C2ARGS" ns1:"--north-star-only --ns-slots 1 --steps 20" ns4:"--north-star-only --ns-slots 4 --steps 20"; do
  name=${d%%:*}; args=${d#*:}
  pass pmc_$name sq "$args" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
  pass pmc_$name fetch "$args" FETCH_SIZE
  pass pmc_$name write "$args" WRITE_SIZE GRBM_GUI_ACTIVE
done
