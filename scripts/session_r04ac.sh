#!/bin/bash
# Round 4: the multi-camera setup stream's priority (-1 product, 0, +1) on the moving frames, and a
# rehearsal of bench.py's N = 2 path (both ranks on this GPU, gloo collectives: plumbing only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04ac
mkdir -p $OUT
TAG=r04ac/ab LIBS="${LIBS:-product mc0 mc1}" ROUNDS=${ROUNDS:-2} CONFIGS=${CONFIGS:-moving_ns,moving_c5} bash scripts/ab_session.sh || exit 1
ERAY_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 4 --warmup 1 > $OUT/rehearsal_n2.json 2> $OUT/rehearsal_n2.err || { tail -30 $OUT/rehearsal_n2.err; exit 1; }
cut -c1-400 $OUT/rehearsal_n2.json
