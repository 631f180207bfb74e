#!/bin/bash
# Masked gather with 32-bit hit words: fused table update timing (+ variants), masked-path parity
# tests, and a short C2 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/pmc_tu.sh KGAT_TU_VARIANT=1 KGAT_TU_VARIANT=5 || exit 1
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "masked or fused_table or hop or frontier or cf_step or propagation or kg_train" > gpurun_out/r03_tu2_parity.log 2>&1; rc=$?
tail -2 gpurun_out/r03_tu2_parity.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/r03_tu2_parity.log | head -20; exit $rc; }
timeout -k 10 600 python -u bench.py --steps 20 --no-cpu-baseline --no-parity --no-kg-leg > gpurun_out/r03_tu2_bench.log 2>&1 || { tail -20 gpurun_out/r03_tu2_bench.log; exit 1; }
python3 -c "
import json; r=json.loads(open('gpurun_out/r03_tu2_bench.log').read().strip().splitlines()[-1])
print('full', r['ms_per_step'], 'frontier', r['frontier_forward']['ms_per_step'], 'tu', r['spmm']['table_update']['avg_launch_ms'], 'fwd', r['spmm']['fwd_avg_ms'])"
