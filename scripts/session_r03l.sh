#!/bin/bash
# Bins pipeline changes: every binned-mesh GPU test, then the moving-camera profiles (C5's frame, 4K/70k).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03l}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_camera_path.py tests/test_gpu_ring.py tests/test_gpu_configs.py tests/test_gpu_trace_binned.py tests/test_gpu_render.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAIL\|Error" $OUT/tests.log | head -80; exit $rc; }
TAG=${TAG:-r03l} bash scripts/prof_moving_r03.sh
