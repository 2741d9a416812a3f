#!/bin/bash
# Round 4: the GPU suite on the product build, the fill-pattern microbenchmark (stream direction,
# RGB / PPM passes, interleaved flat), then product against no fill caps (cap0) on every config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04i}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
if [ $rc -ne 0 ]; then
  grep -B5 -A40 "FAIL\|Error" $OUT/tests.log | head -120
  [ $rc -eq 1 ] || exit $rc  # a crash or a time limit: nothing more on the GPU
fi
timeout -k 10 240 scripts/microbench/fill_pat > $OUT/fill_pat.txt 2>&1 || { cat $OUT/fill_pat.txt; exit 1; }
cat $OUT/fill_pat.txt
TAG=${TAG:-r04i}/ab LIBS="${LIBS:-product cap0}" ROUNDS=${ROUNDS:-2} CONFIGS=${CONFIGS:-aa2,aa_ns,fill4k1,fill4k4,fill8k,fillc2,c2,ns1,ns4,c5,moving_ns,moving_c5} bash scripts/ab_session.sh
