#!/bin/bash
# N=2 bench rehearsal over gloo on one GPU (new test), C4 PMC traffic pass, C5 scaled single-GPU run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "rehearsal" > gpurun_out/rehearsal_tests.log 2>&1; rc=$?
tail -3 gpurun_out/rehearsal_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/rehearsal_tests.log | head -40; exit $rc; }
bash tools/pmc_bench.sh c4 || exit 1
timeout -k 10 400 python -u bench.py --config c5 --scale 0.02 --steps 5 --warmup 2 > gpurun_out/c5_small.log 2>&1 || { tail -20 gpurun_out/c5_small.log; exit 1; }
tail -1 gpurun_out/c5_small.log | cut -c1-300
