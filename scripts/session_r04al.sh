#!/bin/bash
# Round 4, closing: the driver's bench command at HEAD and the N = 2 rehearsal (one GPU, gloo).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04al
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -c 3000 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
ERAY_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 4 --warmup 1 > $OUT/rehearsal_n2.json 2> $OUT/rehearsal_n2.err || { tail -30 $OUT/rehearsal_n2.err; exit 1; }
cut -c1-300 $OUT/rehearsal_n2.json
