#!/bin/bash
# Round 4: the detail waves without the cooperative heavy-bin paths (lt: every sub-block searched
# by its own wave, 139 instead of 161 VGPRs), and C5's separate-fill detail grid at 3 workgroups
# per CU (lt3: light-only; p3: the product build), against the product.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r04am/ab LIBS="${LIBS:-product lt lt3 p3}" ROUNDS=${ROUNDS:-2} CONFIGS=${CONFIGS:-c5,ns1,ns4,c3,moving_ns} bash scripts/ab_session.sh
