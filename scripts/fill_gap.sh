#!/bin/bash
# The frame kernel's empty-scene fill against the plain write stream into the same ring
# (eray_time_write_ceiling), on one box: dispatch-timed A/B (ab_probe.py, alternating), then a
# kernel trace and counter passes of both in one process each (rocprofv3, kernel trace only, one
# pass per counter group).  scripts/pmc_gap_summary.py turns gpurun_out/$TAG into a profile.
#   TAG=r06/fill_gap CONFIGS=fill4k4,ceil4k4 bash scripts/fill_gap.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-fill_gap}
OUT=gpurun_out/$TAG
CONFIGS=${CONFIGS:-fill4k4,ceil4k4}
ABCONFIGS=${ABCONFIGS:-fill4k4,ceil4k4,fill4k1,ceil4k1,fillc2,ceilc2,ns4,ns1}
mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 300 python scripts/ab_probe.py --configs $ABCONFIGS >> $OUT/ab.jsonl 2>> $OUT/ab.err \
    || { tail -20 $OUT/ab.err; exit 1; }
  echo "ab round $r done"
done
run() {  # name rocprofv3-args...
  local name=$1; shift
  echo "=== $name: $*"
  timeout -s KILL 120 rocprofv3 "$@" --kernel-include-regex 'frame_kernel|fill_kernel' --output-format csv \
      -d $OUT/$name -o $name -- python scripts/ab_probe.py --configs $CONFIGS --launches 20 \
      > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/$name.log; exit $rc; fi
}
[ -n "${NO_PMC:-}" ] && exit 0
run stats --kernel-trace --stats
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
run wrreq --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE
run stall --pmc TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_TAG_STALL_sum
run ta --pmc TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum
run write --pmc WRITE_SIZE
