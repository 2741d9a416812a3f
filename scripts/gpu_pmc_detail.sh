#!/bin/bash
# Counter passes over scripts/pmc_detail.py (each pass its own run, kernel trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcd
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex 'frame_kernel' --output-format csv \
      -d gpurun_out/pmcd/$name -o $name -- python scripts/pmc_detail.py > gpurun_out/pmcd/$name.log 2>&1
  local rc=$?
  echo "=== pmc $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/pmcd/$name.log; exit $rc; fi
}
pass a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM
pass b SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
pass c SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES
python scripts/pmc_detail.py report gpurun_out/pmcd
