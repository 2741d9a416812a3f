#!/bin/bash
# Round 4 (data for the next round): the binned meshes' detail share with the per-wave-only build
# (fill workgroups = grid / share: product 2, l175: 1.75, l25: 2.5).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r04ap/ab LIBS="${LIBS:-product l175 l25}" ROUNDS=${ROUNDS:-2} CONFIGS=${CONFIGS:-ns1,ns4,c3} bash scripts/ab_session.sh
