#!/bin/bash
# Dual vs separate wide bi-interaction GEMMs: per-kernel stats and one PMC pass over the dual run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/dual
rm -rf $OUT; mkdir -p $OUT
for v in 0 1; do
  KGAT_DUAL_GEMM=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats$v -o run --output-format csv -- \
    python3 tools/bench_dual.py --rows 300000 > $OUT/b$v.log 2>&1 || { tail -20 $OUT/b$v.log; exit 1; }
  grep '^{' $OUT/b$v.log
done
CTR="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d $OUT/pmc -o run -- \
  python3 tools/bench_dual.py --rows 300000 --reps 3 > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
echo done
