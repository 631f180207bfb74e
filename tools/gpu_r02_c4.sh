#!/bin/bash
# C4 evidence: bench with the extrapolated CPU baseline, then rocprof kernel stats (part=1), or the
# PMC passes for profiles/pmc_c4.json (part=2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${1:-1}" = 1 ]; then
  timeout -k 10 700 python -u bench.py --config c4 --steps 5 --warmup 2 > gpurun_out/r02_c4_bench.log 2>&1 || { tail -20 gpurun_out/r02_c4_bench.log; exit 1; }
  tail -1 gpurun_out/r02_c4_bench.log | cut -c1-300
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
    python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/prof_c4.log 2>&1 || { tail -20 gpurun_out/prof_c4.log; exit 1; }
else
  bash tools/pmc_bench.sh c4
fi
