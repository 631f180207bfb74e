#!/bin/bash
# The 3-layer frontier forward (layer 0 whole, layer 1 on the first hop, layer 2 on the batch rows):
# its bit-identity tests (C2-width and C4-width 3-layer models) + the 3-layer golden tests, then the
# C4 bench (10M nodes / 200M entries, d = 128, [128, 64, 32]) with its frontier leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  tests/test_gpu_parity.py -k "frontier or L3 or large_hub or fused_table or bwd_rows" \
  > gpurun_out/r03_c4fr_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r03_c4fr_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/r03_c4fr_tests.log | head -30; exit $rc; }
timeout -k 10 900 python -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-parity \
  > gpurun_out/r03_c4fr_bench.log 2>&1 || { tail -20 gpurun_out/r03_c4fr_bench.log; exit 1; }
tail -1 gpurun_out/r03_c4fr_bench.log | cut -c1-300
