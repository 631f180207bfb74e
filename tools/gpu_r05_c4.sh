#!/bin/bash
# Round 5: full-size C4 on the current build: the single-GPU step, the sharded DP
# exchange forced at world 1 (RCCL, pipelined owner step), and a kernel trace of the latter (side-stream
# owner Adam + broadcast per block against the backward).  A heartbeat file keeps the long host-side
# graph generation visible as progress.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 50; do date +%T >> gpurun_out/r05_c4_heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
MODE=${1:-lines}
if [ "$MODE" = lines ]; then
  timeout -k 10 560 python -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/r05_c4_bench.log 2>&1 || { tail -30 gpurun_out/r05_c4_bench.log; exit 1; }
  tail -1 gpurun_out/r05_c4_bench.log | cut -c1-300
  timeout -k 10 560 python -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-kg-leg \
    --exchange-at-1 --dp sharded > gpurun_out/r05_c4_exchange_at_1.log 2>&1 || { tail -30 gpurun_out/r05_c4_exchange_at_1.log; exit 1; }
  tail -1 gpurun_out/r05_c4_exchange_at_1.log | cut -c1-300
else
  timeout -k 10 700 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_c4x_trace -o run --output-format csv -- \
    python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-kg-leg --no-frontier-leg \
    --exchange-at-1 --dp sharded > gpurun_out/r05_c4x_trace.log 2>&1 || { tail -30 gpurun_out/r05_c4x_trace.log; exit 1; }
  tail -1 gpurun_out/r05_c4x_trace.log | cut -c1-300
fi
echo done
