#!/bin/bash
# L2 hit/miss per kernel of the C2 bench step (one TCC pass, one TCP pass), plus the counter list.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_l2
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_l2/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc_l2/tcc -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/pmc_l2/tcc.log 2>&1 || { tail -5 gpurun_out/pmc_l2/tcc.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-trace --output-format csv -d gpurun_out/pmc_l2/tcp -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/pmc_l2/tcp.log 2>&1 || { tail -5 gpurun_out/pmc_l2/tcp.log; exit 1; }
echo ok
