#!/bin/bash
# Round-2 end evidence on the final tree: every GPU test + smoke, then the C2 bench (CPU baseline +
# bench-scale parity) and its rocprof kernel stats, and the exchange-overhead rehearsal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/gpu_tests.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r02_c2_bench.log 2>&1 || { tail -20 gpurun_out/r02_c2_bench.log; exit 1; }
tail -1 gpurun_out/r02_c2_bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/prof_c2.log 2>&1 || { tail -20 gpurun_out/prof_c2.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-parity --exchange-at-1 > gpurun_out/r02_c2_exchange_at_1.log 2>&1 || { tail -20 gpurun_out/r02_c2_exchange_at_1.log; exit 1; }
tail -1 gpurun_out/r02_c2_exchange_at_1.log | cut -c1-200
