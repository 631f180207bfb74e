#!/bin/bash
# Quick GPU loop: parity tests, optional kernel microbench section(s), bench (no CPU baseline).
#   bash tools/gpu_quick.sh [bench_kernels sections, e.g. masked,graph]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -15 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
if [ -n "${1:-}" ]; then
  timeout -k 10 300 python tools/bench_kernels.py --only "$1" > gpurun_out/kernels.log 2>&1; rc=$?
  cat gpurun_out/kernels.log | grep kernel
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?
tail -1 gpurun_out/bench.log | cut -c1-900
exit $rc
