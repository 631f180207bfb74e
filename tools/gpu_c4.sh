#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c4.log 2>&1 || { tail -20 gpurun_out/c4.log; exit 1; }
tail -1 gpurun_out/c4.log | cut -c1-420
