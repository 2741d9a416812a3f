#!/bin/bash
# Driver-shaped bench (20 steps) under different warmups and frames per launch: how much of the
# 20-step figure is the first launch's cold start.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/warm
mkdir -p $OUT
for a in ${CASES:-"w5:--warmup 5" "w5b:--warmup 5" "w20:--warmup 20" "w100:--warmup 100" "f4:--warmup 5 --frames-per-launch 4" "f16:--warmup 5 --frames-per-launch 16" "s200:--warmup 20 --steps 200"}; do
  name=${a%%:*}; args=${a#*:}
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 $args --no-cpu-baseline --no-moving-camera > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{')][-1]); print('$name', d['value'], d['ms_per_step']*1e3, d['render_kernel_ms']*1e3, d['config'].get('frames_per_launch'))"
done
