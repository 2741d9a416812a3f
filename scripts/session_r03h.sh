#!/bin/bash
# Binned anti-aliasing: trace tests, then the C3 bench line (with its anti-aliasing line).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03h
mkdir -p $OUT /tmp/eray_meshes
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_trace_binned.py tests/test_gpu_trace.py > $OUT/tests.log 2>&1
rc=$?; tail -30 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o /tmp/eray_meshes/standin70k.obj > /dev/null || exit 1
timeout -k 10 240 python bench.py --mesh /tmp/eray_meshes/standin70k.obj --steps 50 --no-cpu-baseline > $OUT/c3.log 2>&1
rc=$?; grep '^{' $OUT/c3.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d.get('anti_aliased'))); print(d['value'], d.get('moving_camera'))"; exit $rc
