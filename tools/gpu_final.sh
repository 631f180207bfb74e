#!/bin/bash
# KG check + microbench + train-sm profile, then the round's C2 evidence (bench, rocprof, PMC).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_kg_bench.sh || exit $?
bash tools/round_profiles.sh || exit $?
