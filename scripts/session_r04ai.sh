#!/bin/bash
# Round 4: the small-scene fill share at C2 (detail workgroups = grid - grid / share: product 3,
# sh2, sh4, sh6), launch spans per 8-frame launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r04ai/ab LIBS="${LIBS:-product sh2 sh4 sh6}" ROUNDS=${ROUNDS:-3} CONFIGS=${CONFIGS:-c2} bash scripts/ab_session.sh
