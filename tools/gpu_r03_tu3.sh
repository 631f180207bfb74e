#!/bin/bash
# Counters of the fused table update after the 32-bit hit words (tools/pmc_tu.sh with PMC_TU=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
PMC_TU=1 bash tools/pmc_tu.sh
