#!/bin/bash
# Early zero-gradient rows (KGAT_TU_EARLY / KGAT.early_zero_rows): bit-identity tests, then an
# interleaved C2 bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "fused_table or split or early" > gpurun_out/r03_early_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r03_early_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/r03_early_tests.log | head -20; exit $rc; }
for rep in 1 2; do
  for e in 0 1; do
    KGAT_TU_EARLY=$e timeout -k 10 400 python -u bench.py --steps 30 --no-cpu-baseline --no-parity --no-kg-leg \
      > gpurun_out/early_$e.log 2>&1 || { tail -20 gpurun_out/early_$e.log; exit 1; }
    python3 -c "
import json; r=json.loads(open('gpurun_out/early_$e.log').read().strip().splitlines()[-1])
print('early=$e', 'full %.4f' % r['ms_per_step'], 'frontier %.4f' % r['frontier_forward']['ms_per_step'], 'tu(part1) %.4f' % r['spmm']['table_update']['avg_launch_ms'], 'host %.3f' % r['host_launch_ms_per_step'], 'bitid', r['frontier_forward']['bit_identical_to_full']['pass'])"
  done
done
