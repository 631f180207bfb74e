#!/bin/bash
# Round-3 evidence on the current tree: every GPU test + smoke, the C2 bench as the driver runs it
# (CPU baseline, bench-scale parity, KG / refresh legs), its rocprof kernel stats, and the C5 rehearsal
# (2 % scale, world 1, oracle parity).  Each step time-limited; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r03_gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/r03_gpu_tests.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || { tail -20 gpurun_out/r03_smoke.log; exit 1; }
tail -1 gpurun_out/r03_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/r03_c2_bench.log 2>&1 || { tail -20 gpurun_out/r03_c2_bench.log; exit 1; }
tail -1 gpurun_out/r03_c2_bench.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-kg-leg > gpurun_out/r03_prof_c2.log 2>&1 || { tail -20 gpurun_out/r03_prof_c2.log; exit 1; }
timeout -k 10 600 python3 -u bench.py --config c5 --scale 0.02 --steps 8 --warmup 2 > gpurun_out/r03_c5_small_bench.log 2>&1 || { tail -20 gpurun_out/r03_c5_small_bench.log; exit 1; }
tail -1 gpurun_out/r03_c5_small_bench.log | cut -c1-300
