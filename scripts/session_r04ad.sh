#!/bin/bash
# Round 4: wave priorities (s_setprio) of the frame kernel's roles — fill roles and fill_kernel at
# 3 (fp3) or 1 (fp1), detail roles at 3 (dp3) — against the product.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r04ad/ab LIBS="${LIBS:-product fp3 dp3 fp1}" ROUNDS=${ROUNDS:-2} CONFIGS=${CONFIGS:-c2,ns1,ns4,c3,c5,moving_ns} bash scripts/ab_session.sh
