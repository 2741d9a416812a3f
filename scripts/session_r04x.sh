#!/bin/bash
# Round 4: detail claims on cache-line counters (product) and whole-round static deals (bal)
# against the static snake deal (base): the binned configs' GPU tests, then the A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04x}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu_ring.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
if [ $rc -ne 0 ]; then
  grep -B5 -A40 "FAIL\|Error" $OUT/tests.log | head -120
  exit $rc
fi
TAG=${TAG:-r04x}/ab LIBS="${LIBS:-product base bal}" ROUNDS=${ROUNDS:-2} CONFIGS=${CONFIGS:-ns1,ns4,c3,c5,moving_ns} bash scripts/ab_session.sh
