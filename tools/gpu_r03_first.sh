#!/bin/bash
# Round 3, first GPU call: the C5-shape parity tests (single GPU vs the oracle; row-sharded on 2 / 4
# ranks vs single-GPU KGAT), then the C5 rehearsal (2 % scale, world 1) under rocprofv3 --stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_sharded.py -k "256 or sharded_ranks or extra_table or id_error_raised" > gpurun_out/r03_c5_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r03_c5_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/r03_c5_tests.log | head -40; exit $rc; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- \
  python3 bench.py --config c5 --scale 0.02 --steps 8 --warmup 2 > gpurun_out/r03_c5_prof.log 2>&1; rc=$?
tail -1 gpurun_out/r03_c5_prof.log | cut -c1-400
exit $rc
