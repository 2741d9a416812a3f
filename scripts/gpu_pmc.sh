#!/bin/bash
# rocprofv3 counter passes for the render kernel (each pass its own run, kernel trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${PMC_DIR:-pmc}  # output directory under gpurun_out/
mkdir -p gpurun_out/$D
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 50 --warmup 5 --no-cpu-baseline --no-moving-camera}
pass() {  # name counters...
  local name=$1; shift
  echo "=== pmc $name: $*"
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex 'frame_kernel|fill_kernel' \
      --output-format csv -d gpurun_out/$D/$name -o $name -- python bench.py $ARGS \
      > gpurun_out/$D/$name.log 2>&1
  local rc=$?
  echo "=== pmc $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/$D/$name.log; exit $rc; fi
}
pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
pass fetch FETCH_SIZE
pass write WRITE_SIZE GRBM_GUI_ACTIVE
