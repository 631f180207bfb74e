#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/host_profile.py --kg --lazy > gpurun_out/hp_kg_lazy.log 2>&1 || { tail -20 gpurun_out/hp_kg_lazy.log; exit 1; }
timeout -k 10 300 python3 tools/host_profile.py > gpurun_out/hp_frontier.log 2>&1 || { tail -20 gpurun_out/hp_frontier.log; exit 1; }
grep -h "ms/step" gpurun_out/hp_kg_lazy.log gpurun_out/hp_frontier.log
