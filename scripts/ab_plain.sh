#!/bin/bash
# A/B on one box: the driver's bench command with the frame loop replayed from HIP graphs (default)
# or launched directly (ERAY_PLAIN_LAUNCHES=1), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_plain
mkdir -p $OUT
for rep in 1 2 3; do
  for mode in graph plain; do
    if [ $mode = plain ]; then export ERAY_PLAIN_LAUNCHES=1; else unset ERAY_PLAIN_LAUNCHES; fi
    timeout -k 10 120 python3 bench.py --gpus 1 --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-moving-camera > $OUT/$mode$rep.log 2>&1 || { tail -5 $OUT/$mode$rep.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$OUT/$mode$rep.log') if l.startswith('{')][-1]); print('$mode$rep', d['value'], round(d['ms_per_step']*1e3,3), round(d['render_kernel_ms']*1e3,3))"
  done
done
