#!/bin/bash
# Round 4, final: the GPU suite, the driver's bench command and its per-leg rocprof rows at HEAD
# (north-star kernel over 64 launches); counters unchanged since r04z (same kernels).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
NO_PMC=1 TAG=${TAG:-r04af} bash scripts/session_r04z.sh
