#!/bin/bash
# Round 4: cameras per multi-camera build (16, product; 8; 4) on the moving 70k frame.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r04aa}/ab LIBS="${LIBS:-product k8 k4}" ROUNDS=${ROUNDS:-2} CONFIGS=${CONFIGS:-moving_ns,moving_c5} bash scripts/ab_session.sh
