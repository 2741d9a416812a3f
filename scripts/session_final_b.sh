#!/bin/bash
# Final validation at HEAD after the last kernel changes: the whole GPU suite, smoke, the driver's
# bench command, then the moving-camera profiles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-final_b}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -B2 -A40 "FAILED\|Error" $OUT/tests.log | head -120; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.log 2>&1 || { tail -20 $OUT/bench20.log; exit 1; }
grep '^{' $OUT/bench20.log | tail -1 > $OUT/bench20.json
python -c "import json; d=json.load(open('$OUT/bench20.json')); print('bench20', d['value'], d['ms_per_step'], d['roofline']['frac'], 'moving', d['moving_camera']['frame_ms'])"
TAG=${TAG:-final_b} bash scripts/prof_moving_r03.sh
