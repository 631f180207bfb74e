#!/bin/bash
# Round 3: the all-peer row-sharded path (sharded.py) and the fused KG table update on the GPU --
# every sharded / DP / RCCL test and the new parity tests, then the C5 rehearsal (2 % scale, world 1,
# parity vs the oracle) under rocprofv3 --stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  tests/test_gpu_sharded.py tests/test_gpu_parity.py -k "sharded or dp_ or rccl or rehearsal or kg_table or extra_table or id_error or kg_step" \
  > gpurun_out/r03_sharded_tests.log 2>&1; rc=$?
tail -25 gpurun_out/r03_sharded_tests.log
grep -h "sharded parity ok" gpurun_out/sharded_world*.log | head -8
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/r03_sharded_tests.log | head -40; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5n -o run --output-format csv -- \
  python3 bench.py --config c5 --scale 0.02 --steps 8 --warmup 2 > gpurun_out/r03_c5n_prof.log 2>&1; rc=$?
tail -1 gpurun_out/r03_c5n_prof.log | cut -c1-600
exit $rc
