#!/bin/bash
# Round 4: frames in flight on one or two streams (scripts/dual_probe.py), after the ring tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04y}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ring.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { grep -B5 -A40 "FAIL\|Error" $OUT/tests.log | head -80; exit $rc; }
for r in 1 2; do
  timeout -k 10 300 python scripts/dual_probe.py 2>&1 | grep -v amdgpu.ids | tee -a $OUT/dual.jsonl || exit 1
done
# the moving-camera 70k frame's kernels (setup chain beside the frames)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_moving_ns -o run -- python3 scripts/ab_probe.py --configs moving_ns > $OUT/moving_ns.json 2> $OUT/moving_ns.err || { tail -20 $OUT/moving_ns.err; exit 1; }
cat $OUT/moving_ns.json
