#!/bin/bash
# Fused table update with the row blocks in a strided order (KGAT_TU_PERM): microbench + digest, then an
# interleaved C2 bench A/B; the driver test (lazy KG Adam now on in driver.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_tu.sh KGAT_TU_PERM=1 || exit 1
for v in 0 1; do KGAT_SPMM_PERM=$v timeout -k 10 300 python3 tools/bench_kernels.py --only spmm --reps 20 > gpurun_out/spmm_perm.log 2>&1 || exit 1; echo "SPMM_PERM=$v"; grep spmm_fwd gpurun_out/spmm_perm.log; done
for rep in 1 2; do
  for e in 0 1; do
    KGAT_TU_PERM=$e timeout -k 10 400 python -u bench.py --steps 30 --no-cpu-baseline --no-parity --no-kg-leg \
      > gpurun_out/perm_$e.log 2>&1 || { tail -20 gpurun_out/perm_$e.log; exit 1; }
    python3 -c "
import json; r=json.loads(open('gpurun_out/perm_$e.log').read().strip().splitlines()[-1])
print('perm=$e', 'full %.4f' % r['ms_per_step'], 'frontier %.4f' % r['frontier_forward']['ms_per_step'], 'tu %.4f' % r['spmm']['table_update']['avg_launch_ms'], 'bitid', r['frontier_forward']['bit_identical_to_full']['pass'])"
  done
done
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "driver or lazy" > gpurun_out/r03_driver_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r03_driver_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/r03_driver_tests.log | head -20; exit $rc; }
exit 0
