#!/bin/bash
# Material::update's kernel (shaderlib.hip material_example_kernel, main.rs's graph on a 1024 x 1024
# texture) under rocprofv3: kernel-trace statistics, then counter passes (each its own run, kernel
# trace only).  scripts/mat_pmc_summary.py turns gpurun_out/$D into profiles/.
#   bash scripts/mat_pmc.sh            (ERAY_LIB selects a library build, as for ab_probe.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${PMC_DIR:-mat_pmc}
mkdir -p gpurun_out/$D
export TMPDIR=/tmp
run() {  # name rocprofv3-args...
  local name=$1; shift
  echo "=== $name: $*"
  timeout -k 10 300 rocprofv3 "$@" --kernel-include-regex 'material_example_kernel' --output-format csv \
      -d gpurun_out/$D/$name -o $name -- python scripts/ab_probe.py --configs mat > gpurun_out/$D/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/$D/$name.log; exit $rc; fi
}
run stats --kernel-trace --stats
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
run write --pmc WRITE_SIZE GRBM_GUI_ACTIVE
run valu --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_ANY
