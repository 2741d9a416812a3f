#!/bin/bash
# Round 4: the multi-camera build size A/B (16 / 8 / 4 cameras per chain), camera-path frames of
# the scene camera against its static frames (frame kernel durations), then the round's profiles
# at the product (scripts/session_r04z.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/session_r04aa.sh || exit 1
OUT=gpurun_out/r04ab
mkdir -p $OUT
for m in static still dolly; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$m -o run -- python3 scripts/path_still_probe.py --mode $m > $OUT/$m.json 2> $OUT/$m.err || { tail -20 $OUT/$m.err; exit 1; }
  cat $OUT/$m.json
done
TAG=r04z bash scripts/session_r04z.sh
