#!/bin/bash
# Round 4, first GPU check: the new / changed tests (ADVICE r3 lazy-Adam cases, C4-shape DP exchange
# at worlds 2 / 4, the C4 gloo bench rehearsal), then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -v -p no:cacheprovider \
  --timeout 600 --timeout-method thread -k "gloo_rehearsal or sharded_ranks" > gpurun_out/r04_first_tests.log 2>&1 \
  || { grep -E "^E |FAILED|PASSED" gpurun_out/r04_first_tests.log | head -40; tail -3 gpurun_out/r04_first_tests.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r04_first_tests.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/r04_first_all.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r04_first_all.log | head -30; tail -3 gpurun_out/r04_first_all.log; exit 1; }
tail -1 gpurun_out/r04_first_all.log
