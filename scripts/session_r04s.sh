#!/bin/bash
# Round 4: every frame in device-camera mode (dev: the setup's CamState read by the kernels) against
# args mode (product) — C5's first, device-camera frame measured 131 us against 147-150 in args mode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r04s}/ab LIBS="product dev" ROUNDS=2 CONFIGS=c5,ns1,ns4,c3,c2 bash scripts/ab_session.sh
