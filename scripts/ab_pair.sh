#!/bin/bash
# A/B of HEAD against the build tree ab_base/ on C3 and 3840x2160 / 70k (static frames), after the
# GPU tests (SKIP_TESTS=1 skips them).  Every GPU step has its own limit; a failure ends the run.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
      -p no:cacheprovider > gpurun_out/ab_pytest.log 2>&1 || { tail -20 gpurun_out/ab_pytest.log; exit 1; }
  tail -2 gpurun_out/ab_pytest.log
fi
AB_TREES="head base" AB_ARGS='--mesh $M/standin70k.obj --width 3840 --height 2160 --steps 200 --warmup 20' \
  bash scripts/ab_config.sh || exit 1
AB_TREES="head base" AB_ARGS='--mesh $M/standin70k.obj --steps 400 --warmup 40' bash scripts/ab_config.sh || exit 1
