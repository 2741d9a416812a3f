#!/bin/bash
# Round 4: the GPU suite on the product build, one probe pass over every config (launch spans),
# and a kernel trace of the moving-camera paths (C5, 3840x2160 / 70k).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04l}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
if [ $rc -ne 0 ]; then
  grep -B5 -A40 "FAIL\|Error" $OUT/tests.log | head -120
  [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 300 python scripts/ab_probe.py --configs aa2,aa_ns,fill4k1,fill4k4,fill8k,fillc2,c2,ns1,ns4,c5,moving_ns,moving_c5 > $OUT/probe.json 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
cat $OUT/probe.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/moving -o run -- python3 $GRAFT_REPO_ROOT/scripts/ab_probe.py --configs moving_c5,moving_ns > $GRAFT_REPO_ROOT/$OUT/moving.log 2>&1
rc=$?; tail -3 $GRAFT_REPO_ROOT/$OUT/moving.log; exit $rc
