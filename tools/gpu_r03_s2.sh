#!/bin/bash
# Round 3, second session: the whole -m gpu suite on this tree, the C2 bench (CPU baseline, KG and
# refresh legs), the C5 rehearsal (2 % scale, world 1, all-peer gather path) under rocprofv3 --stats,
# then the C5 rehearsal's FETCH_SIZE / WRITE_SIZE passes (profiles/pmc_c5.json).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/r03_gpu_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r03_gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/r03_gpu_tests.log | head -40; exit $rc; }
timeout -k 10 600 python -u bench.py > gpurun_out/r03_c2_bench.log 2>&1 || { tail -20 gpurun_out/r03_c2_bench.log; exit 1; }
tail -1 gpurun_out/r03_c2_bench.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- \
  python3 bench.py --config c5 --scale 0.02 --steps 8 --warmup 2 > gpurun_out/r03_c5_prof.log 2>&1 || { tail -20 gpurun_out/r03_c5_prof.log; exit 1; }
tail -1 gpurun_out/r03_c5_prof.log | cut -c1-300
bash tools/pmc_bench.sh c5 --scale 0.02
