#!/bin/bash
# Round 3: the whole -m gpu suite (lazy KG Adam, sharded fused table update and everything before),
# the C2 bench (KG legs timed without per-kernel events; lazy KG leg), the C5 rehearsal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/r03_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r03_gpu_tests.log
grep -h "bit-identical" gpurun_out/sharded_world*.log | head -4
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/r03_gpu_tests.log | head -40; exit $rc; }
timeout -k 10 600 python -u bench.py > gpurun_out/r03_c2_bench.log 2>&1 || { tail -20 gpurun_out/r03_c2_bench.log; exit 1; }
tail -1 gpurun_out/r03_c2_bench.log | cut -c1-200
timeout -k 10 600 python -u bench.py --config c5 --scale 0.02 --steps 8 --warmup 2 > gpurun_out/r03_c5_bench.log 2>&1 \
  || { tail -20 gpurun_out/r03_c5_bench.log; exit 1; }
tail -1 gpurun_out/r03_c5_bench.log | cut -c1-200
