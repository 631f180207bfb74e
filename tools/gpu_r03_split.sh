#!/bin/bash
# The fused table update split in two row launches (KGAT_TU_SPLIT): microbench + digest, the new
# bit-identity tests, and an interleaved C2 bench A/B of the split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_tu.sh KGAT_TU_SPLIT=1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "fused_table or split" > gpurun_out/r03_split_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r03_split_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/r03_split_tests.log | head -20; exit $rc; }
for rep in 1 2; do
  for sp in 0 1; do
    KGAT_TU_SPLIT=$sp timeout -k 10 400 python -u bench.py --steps 30 --no-cpu-baseline --no-parity --no-kg-leg \
      > gpurun_out/split_$sp.log 2>&1 || { tail -20 gpurun_out/split_$sp.log; exit 1; }
    python3 -c "
import json; r=json.loads(open('gpurun_out/split_$sp.log').read().strip().splitlines()[-1])
print('split=$sp', 'full %.4f' % r['ms_per_step'], 'frontier %.4f' % r['frontier_forward']['ms_per_step'], 'tu %.4f' % r['spmm']['table_update']['avg_launch_ms'], 'bitid', r['frontier_forward']['bit_identical_to_full']['pass'])"
  done
done
