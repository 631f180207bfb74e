#!/bin/bash
# C4 on the round-3 final build (full + frontier step, fused table update), with rocprof kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-parity \
  > gpurun_out/r03_c4_final_bench.log 2>&1 || { tail -20 gpurun_out/r03_c4_final_bench.log; exit 1; }
tail -1 gpurun_out/r03_c4_final_bench.log | cut -c1-300
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
  python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-kg-leg > gpurun_out/r03_prof_c4.log 2>&1 || { tail -20 gpurun_out/r03_prof_c4.log; exit 1; }
