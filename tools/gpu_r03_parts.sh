#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TU_PARTS=1 timeout -k 10 300 python3 tools/bench_tu.py --tag parts > gpurun_out/tu_parts.log 2>&1 || { tail -20 gpurun_out/tu_parts.log; exit 1; }
tail -1 gpurun_out/tu_parts.log
