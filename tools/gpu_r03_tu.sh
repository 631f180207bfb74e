#!/bin/bash
# Fused table update variants (KGAT_TU_VARIANT) at C2 + SQ counters of the default kernel; the
# bi-interaction forward at 64->64 (KGAT_FWD_VARIANT 8 / 12) after the DPP row sums; parity tests of
# the kernels that use the row sums.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
PMC_TU=1 bash tools/pmc_tu.sh KGAT_TU_VARIANT=1 KGAT_TU_VARIANT=2 KGAT_TU_VARIANT=3 KGAT_TU_VARIANT=4 KGAT_TU_VARIANT=5 KGAT_TU_VARIANT=6 KGAT_TU_BATCH=1 || exit 1
for v in 8 12 0 20; do
  KGAT_FWD_VARIANT=$v timeout -k 10 300 python3 tools/bench_kernels.py --only graph --reps 10 > gpurun_out/fwd_v$v.log 2>&1 || { tail -5 gpurun_out/fwd_v$v.log; exit 1; }
  echo "FWD_VARIANT=$v"; grep '"biinter_fwd_' gpurun_out/fwd_v$v.log | cut -c1-150
done
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "biinter or attention or fused_table or cf_step or propagation or frontier_forward_bit" > gpurun_out/r03_s3_parity.log 2>&1; rc=$?
tail -2 gpurun_out/r03_s3_parity.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/r03_s3_parity.log | head -20; exit $rc; }
exit 0
