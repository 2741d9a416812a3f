#!/bin/bash
# Round 4: light sub-block search for every sub-block of a binned object (ltr: the cooperative
# heavy-bin path off at run time when the frame has a detail list and bins; lt: the cooperative
# paths compiled out) against the product.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r04an/ab LIBS="${LIBS:-product ltr lt}" ROUNDS=${ROUNDS:-2} CONFIGS=${CONFIGS:-ns1,ns4,c3,c5,moving_ns,moving_c5,c2} bash scripts/ab_session.sh
