#!/bin/bash
# Round 4: the GPU suite on the product build (64-B bin entries), then a same-box A/B against the
# previous commit (pre: three entry arrays, setup stream at normal priority).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04q}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
if [ $rc -ne 0 ]; then
  grep -B5 -A40 "FAIL\|Error" $OUT/tests.log | head -120
  exit $rc
fi
TAG=${TAG:-r04q}/ab LIBS="${LIBS:-product pre}" ROUNDS=${ROUNDS:-2} CONFIGS=${CONFIGS:-c3,ns1,ns4,c5,aa_ns,moving_c5,moving_ns} bash scripts/ab_session.sh
