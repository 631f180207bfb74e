#!/bin/bash
# Full GPU test suite + smoke + C2 bench (30 steps) + C4 bench with rocprof stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/gpu_tests.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/bench_c2.log 2>&1 || { tail -20 gpurun_out/bench_c2.log; exit 1; }
tail -1 gpurun_out/bench_c2.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
  python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/bench_c4.log 2>&1 || { tail -20 gpurun_out/bench_c4.log; exit 1; }
timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/bench_c4_noprof.log 2>&1 || { tail -20 gpurun_out/bench_c4_noprof.log; exit 1; }
tail -1 gpurun_out/bench_c4_noprof.log | cut -c1-300
