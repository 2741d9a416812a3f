#!/bin/bash
# One scripts/ab_probe.py configuration under rocprofv3: kernel-trace statistics, then counter
# passes (each its own run, kernel trace only) for the frame kernel (and the separate fill kernel).
# scripts/probe_pmc_summary.py turns gpurun_out/$D into profiles/.
#   CONFIG=c5s3 PMC_DIR=pmc_c5s3 bash scripts/probe_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CONFIG=${CONFIG:-c5s3}
D=${PMC_DIR:-pmc_$CONFIG}
mkdir -p gpurun_out/$D
export TMPDIR=/tmp
run() {  # name rocprofv3-args...
  local name=$1; shift
  echo "=== $name: $*"
  timeout -k 10 300 rocprofv3 "$@" --kernel-include-regex 'frame_kernel|fill_kernel' --output-format csv \
      -d gpurun_out/$D/$name -o $name -- python scripts/ab_probe.py --configs $CONFIG --launches 20 \
      > gpurun_out/$D/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/$D/$name.log; exit $rc; fi
}
run stats --kernel-trace --stats
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE GRBM_GUI_ACTIVE
