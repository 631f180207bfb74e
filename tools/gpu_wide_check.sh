#!/bin/bash
# Full GPU parity suite, then the wide-layer microbench (bits vs gemm state).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -4 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_kernels.py --only wide --reps 10 > gpurun_out/wide.log 2>&1 || { tail -20 gpurun_out/wide.log; exit 1; }
grep kernel gpurun_out/wide.log
