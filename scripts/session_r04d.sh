#!/bin/bash
# Round 4: binned-mesh GPU tests on the current build, then a same-box A/B against the base build,
# then the diagnostics of session_r04c.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04d}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_ring.py tests/test_gpu_camera_path.py tests/test_gpu_render.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAIL\|Error" $OUT/tests.log | head -150; exit $rc; }
TAG=${TAG:-r04d}/ab LIBS="base product" ROUNDS=2 CONFIGS=${CONFIGS:-c2,c3,ns1,ns4} bash scripts/ab_session.sh || exit 1
[ "${DIAG:-1}" = 1 ] && TAG=${TAG:-r04d}/diag bash scripts/session_r04c.sh
