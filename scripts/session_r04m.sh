#!/bin/bash
# Round 4: (1) the binned meshes' detail share (sh15 / sh3 / sh4: grid / 1.5, 3, 4 fill workgroups
# against the product's grid / 2); (2) the multi-camera setup stream (pri; pri2: and the separate
# fill's) at another priority so that HIP gives it its own hardware queue (on one queue with the
# frames' stream they serialise); then a kernel trace of the moving C5 path under pri.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04m}
mkdir -p $OUT
export TMPDIR=/tmp
TAG=${TAG:-r04m}/share LIBS="product sh15 sh3 sh4" ROUNDS=2 CONFIGS=ns1,ns4,c3,c5 bash scripts/ab_session.sh || exit 1
TAG=${TAG:-r04m}/pri LIBS="product pri pri2" ROUNDS=2 CONFIGS=moving_c5,moving_ns,c5 bash scripts/ab_session.sh || exit 1
cd /tmp && ERAY_LIB=$GRAFT_REPO_ROOT/eray_amd/lib/liberay_hip_pri.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/moving_pri -o run -- python3 $GRAFT_REPO_ROOT/scripts/ab_probe.py --configs moving_c5 > $GRAFT_REPO_ROOT/$OUT/moving_pri.log 2>&1
rc=$?; tail -2 $GRAFT_REPO_ROOT/$OUT/moving_pri.log; exit $rc
