#!/bin/bash
# Round 4, final bench line and its per-leg rocprof rows at HEAD (GPU suite: r04af, same product).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04ah
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; [ $rc -eq 0 ] || { tail -c 3000 $OUT/bench.err; exit $rc; }
cut -c1-300 $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err
rc=$?; [ $rc -eq 0 ] || { tail -c 3000 $OUT/bench_prof.err; exit $rc; }
