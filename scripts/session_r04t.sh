#!/bin/bash
# Round 4: the GPU suite on the product build (split heavy-first detail lists for camera paths),
# then the moving-camera configs against the previous commit (pre).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04t}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
if [ $rc -ne 0 ]; then
  grep -B5 -A40 "FAIL\|Error" $OUT/tests.log | head -120
  exit $rc
fi
TAG=${TAG:-r04t}/ab LIBS="${LIBS:-product pre}" ROUNDS=${ROUNDS:-2} CONFIGS=${CONFIGS:-moving_ns,moving_c5,ns1} bash scripts/ab_session.sh
