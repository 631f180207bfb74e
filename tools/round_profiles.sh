#!/bin/bash
# Round-end evidence on one GPU: bench (with the CPU baseline), rocprof kernel stats of the
# bench, and the forward SpMM's HBM traffic (PMC, tools/pmc_spmm.sh).  Each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_round -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_round.log 2>&1 || { tail -20 gpurun_out/prof_round.log; exit 1; }
bash tools/pmc_spmm.sh
