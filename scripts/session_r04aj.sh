#!/bin/bash
# Round 4: the frame kernel's fill roles start late (s_sleep ~1.3 us: fd1, ~3.4 us: fd3), so the
# detail waves' first round meets a quieter memory system, against the product.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r04aj/ab LIBS="${LIBS:-product fd1 fd3}" ROUNDS=${ROUNDS:-2} CONFIGS=${CONFIGS:-ns1,ns4,c2,c3,moving_ns} bash scripts/ab_session.sh
