#!/bin/bash
# Round 4: the GPU suite on the product build (per-wave detail claims after the first round,
# rotating gather roots), the binned configs against the previous frame kernel (base), then the
# driver's bench command (a step = one batch of frames).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04w}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
if [ $rc -ne 0 ]; then
  grep -B5 -A40 "FAIL\|Error" $OUT/tests.log | head -120
  exit $rc
fi
TAG=${TAG:-r04w}/ab LIBS="${LIBS:-product base}" ROUNDS=${ROUNDS:-2} CONFIGS=${CONFIGS:-ns1,ns4,c3,c5,moving_ns,moving_c5} bash scripts/ab_session.sh || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print({k:d[k] for k in ('value','ms_per_step','frame_ms','render_kernel_ms')}, d['north_star'] and {k:v for k,v in d['north_star'].items() if not isinstance(v,(dict,list))})"
