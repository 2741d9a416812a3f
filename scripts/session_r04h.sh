#!/bin/bash
# Round 4: the GPU suite on the product build (fill workgroups capped at one per CU), then
# same-box A/Bs: the fill cap (cap0: none, cap2: two per CU) against HEAD (pf) on every config,
# and the tracer steps (t0, t1) on the anti-aliasing configs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04h}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
if [ $rc -ne 0 ]; then
  grep -B5 -A40 "FAIL\|Error" $OUT/tests.log | head -120
  [ $rc -eq 1 ] || exit $rc  # a crash or a time limit: nothing more on the GPU
fi
TAG=${TAG:-r04h}/aa LIBS="product t0 t1" ROUNDS=2 CONFIGS=aa2,aa_ns bash scripts/ab_session.sh || exit 1
TAG=${TAG:-r04h}/ab LIBS="${LIBS:-product cap0 cap2 pf}" ROUNDS=${ROUNDS:-2} CONFIGS=${CONFIGS:-fill4k1,fill4k4,fill8k,fillc2,c2,ns1,ns4,c5,moving_ns,moving_c5} bash scripts/ab_session.sh
