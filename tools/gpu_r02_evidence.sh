#!/bin/bash
# Round-2 evidence on the current build: GPU tests + smoke, PMC passes of the C2 bench
# (profiles/pmc_c2.json: forward SpMM + fused table update), the C2 bench with CPU baseline and
# bench-scale parity, rocprof stats of C2, C4 bench (extrapolated CPU baseline) and C4 rocprof stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/gpu_tests.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/pmc_bench.sh c2 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r02_c2_bench.log 2>&1 || { tail -20 gpurun_out/r02_c2_bench.log; exit 1; }
tail -1 gpurun_out/r02_c2_bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/prof_c2.log 2>&1 || { tail -20 gpurun_out/prof_c2.log; exit 1; }
timeout -k 10 900 python -u bench.py --config c4 --steps 5 --warmup 2 > gpurun_out/r02_c4_bench.log 2>&1 || { tail -20 gpurun_out/r02_c4_bench.log; exit 1; }
tail -1 gpurun_out/r02_c4_bench.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
  python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/prof_c4.log 2>&1 || { tail -20 gpurun_out/prof_c4.log; exit 1; }
