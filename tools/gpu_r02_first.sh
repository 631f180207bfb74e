#!/bin/bash
# Round-2 first GPU trip: GPU tests, smoke, full bench (CPU baseline + bench-scale parity), rocprof
# kernel stats of the bench, PMC traffic over the bench, a C5-shaped row-sharded rehearsal on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -4 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/prof_c2.log 2>&1 || { tail -20 gpurun_out/prof_c2.log; exit 1; }
bash tools/pmc_bench.sh c2 || exit 1
timeout -k 10 400 python -u bench.py --config c5 --scale 0.02 --steps 5 --warmup 2 > gpurun_out/c5_small.log 2>&1 || { tail -20 gpurun_out/c5_small.log; exit 1; }
tail -1 gpurun_out/c5_small.log | cut -c1-400
