#!/bin/bash
# Round-3 final check at HEAD: the whole GPU suite, smoke, the driver's bench command and its
# rocprofv3 kernel statistics.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/final_a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -B2 -A40 "FAILED\|Error" $OUT/tests.log | head -120; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.log 2>&1 || { tail -20 $OUT/bench20.log; exit 1; }
grep '^{' $OUT/bench20.log | tail -1 > $OUT/bench20.json
python -c "import json; d=json.load(open('$OUT/bench20.json')); print('bench20', d['value'], d['ms_per_step'], d['roofline']['frac'], 'moving', d['moving_camera']['frame_ms'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
