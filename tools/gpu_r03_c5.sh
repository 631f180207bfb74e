#!/bin/bash
# Round 3: the all-peer row-sharded path, the fused KG table update, the k-major GEMM LDS layout on the
# GPU -- the sharded / DP / RCCL tests and the new parity tests; then the C2 bench with its KG /
# refresh legs; an A/B of the row-batched fused table update (KGAT_TU_BATCH=1); the C5 rehearsal
# (2 % scale, world 1, parity vs the oracle) under rocprofv3 --stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  tests/test_gpu_gemm.py tests/test_gpu_sharded.py tests/test_gpu_parity.py \
  -k "gemm or sharded or dp_ or rccl or rehearsal or kg_table or extra_table or id_error or kg_step or biinter_wide" \
  > gpurun_out/r03_sharded_tests.log 2>&1; rc=$?
tail -30 gpurun_out/r03_sharded_tests.log
grep -h "sharded parity ok" gpurun_out/sharded_world*.log | head -12
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/r03_sharded_tests.log | head -40; exit $rc; }
timeout -k 10 600 python -u bench.py > gpurun_out/r03_c2_bench.log 2>&1 || { tail -20 gpurun_out/r03_c2_bench.log; exit 1; }
tail -1 gpurun_out/r03_c2_bench.log | cut -c1-400
for v in 0 1 0 1; do
  KGAT_TU_BATCH=$v timeout -k 10 300 python -u bench.py --steps 30 --no-cpu-baseline --no-parity --no-kg-leg \
    > gpurun_out/r03_tu_ab_$v.log 2>&1 || { tail -20 gpurun_out/r03_tu_ab_$v.log; exit 1; }
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/r03_tu_ab_$v.log').read().strip().splitlines()[-1]); print('TU_BATCH=$v', r['ms_per_step'], r['frontier_forward']['ms_per_step'], r['spmm']['table_update']['avg_launch_ms'])"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5n -o run --output-format csv -- \
  python3 bench.py --config c5 --scale 0.02 --steps 8 --warmup 2 > gpurun_out/r03_c5n_prof.log 2>&1; rc=$?
tail -1 gpurun_out/r03_c5n_prof.log | cut -c1-600
exit $rc
