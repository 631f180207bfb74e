#!/bin/bash
# Session-3 entry check: the -m gpu suite on the rebuilt library, then the round-3 MFMA PMC pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/r03_gpu_tests_s3.log 2>&1; rc=$?
tail -2 gpurun_out/r03_gpu_tests_s3.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/r03_gpu_tests_s3.log | head -30; exit $rc; }
bash tools/pmc_mfma_r03.sh
