#!/bin/bash
# Round 3: the row-sharded tests (worlds 1/2/4, C2 and C5 shapes) and the C5 rehearsal bench
# (2 % scale, world 1, parity vs the oracle) with its kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  tests/test_gpu_sharded.py -k "sharded or rehearsal or rccl" > gpurun_out/r03_shard_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r03_shard_tests.log
grep -h "bit-identical" gpurun_out/sharded_world*.log | head -12
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error|FAIL" gpurun_out/r03_shard_tests.log | head -40; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5b -o run --output-format csv -- \
  python3 bench.py --config c5 --scale 0.02 --steps 8 --warmup 2 > gpurun_out/r03_c5b.log 2>&1 || { tail -20 gpurun_out/r03_c5b.log; exit 1; }
tail -1 gpurun_out/r03_c5b.log | cut -c1-400
