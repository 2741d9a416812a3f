#!/bin/bash
# Round 4, final product (culled large-mesh builds without the cooperative paths): smoke, the GPU
# suite, the driver's bench command and its per-leg rocprof rows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04ao
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAIL\|Error" $OUT/tests.log | head -100; exit $rc; }
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -c 3000 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -c 3000 $OUT/bench_prof.err; exit 1; }
TAG=r04ao/ab LIBS=product ROUNDS=1 CONFIGS=c5,moving_ns,moving_c5 bash scripts/ab_session.sh
