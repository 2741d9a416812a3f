#!/bin/bash
# Round 4: cameras per multi-camera build at a million faces (product 4; c5k8: 8; c5k2: 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r04ae/ab LIBS="${LIBS:-product c5k8 c5k2}" ROUNDS=${ROUNDS:-2} CONFIGS=${CONFIGS:-moving_c5} bash scripts/ab_session.sh
