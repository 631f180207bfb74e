#!/bin/bash
# C4 single-GPU step: tests of the wide path, a short bench, rocprof kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "gemm or wide or d128 or d256 or dense_backward" > gpurun_out/c4_tests.log 2>&1; rc=$?
tail -2 gpurun_out/c4_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/c4_tests.log | head -30; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
  python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/bench_c4.log 2>&1 || { tail -20 gpurun_out/bench_c4.log; exit 1; }
timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/bench_c4_noprof.log 2>&1 || { tail -20 gpurun_out/bench_c4_noprof.log; exit 1; }
tail -1 gpurun_out/bench_c4_noprof.log | cut -c1-400
