#!/bin/bash
# GEMM + wide-layer checks and microbench, then a short C2 bench (no CPU leg).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -4 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/gpu_tests.log | head -30; exit $rc; }
timeout -k 10 300 python -u tools/bench_kernels.py --only gemm,wide --reps 10 > gpurun_out/gemm_bench.log 2>&1 || { tail -20 gpurun_out/gemm_bench.log; exit 1; }
cat gpurun_out/gemm_bench.log | grep kernel
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/bench_quick.log 2>&1 || { tail -20 gpurun_out/bench_quick.log; exit 1; }
tail -1 gpurun_out/bench_quick.log | cut -c1-300
