#!/bin/bash
# Round 4: the north-star frame with the separate flat-order fill (ns*sep) against the single
# launch (ns1, ns4), and more binned-tracer light workgroups (lw8) on the AA configs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r04k}/ab LIBS="${LIBS:-product lw8}" ROUNDS=${ROUNDS:-2} CONFIGS=${CONFIGS:-aa_ns,aa2,ns1,ns1sep,ns4,ns4sep,c5} bash scripts/ab_session.sh
