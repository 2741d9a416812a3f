#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a crash/timeout/fault (rc >= 124 or signal) stops the
# session, test failures (rc 1) do not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-200}
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "stopping after $name (rc=$rc)"; exit $rc
  fi
  return 0
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  run pytest_gpu 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
run bench 600 python bench.py --steps "$STEPS" --warmup 20 --cpu-seconds 10
if [ "${SKIP_PROF:-0}" != 1 ]; then
  run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline
fi
