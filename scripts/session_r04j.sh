#!/bin/bash
# Round 4: the GPU suite on the product build (flat-order separate fill), then a same-box A/B
# against the block-order fill (noflat) and the freed fill workgroups given to detail (dw).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04j}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
if [ $rc -ne 0 ]; then
  grep -B5 -A40 "FAIL\|Error" $OUT/tests.log | head -120
  [ $rc -eq 1 ] || exit $rc  # a crash or a time limit: nothing more on the GPU
fi
TAG=${TAG:-r04j}/ab LIBS="${LIBS:-product noflat dw}" ROUNDS=${ROUNDS:-2} CONFIGS=${CONFIGS:-fillc2,c2,ns1,ns4,c5,moving_c5} bash scripts/ab_session.sh
