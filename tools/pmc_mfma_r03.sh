#!/bin/bash
# Round-3 MFMA utilisation pass: the C2 bi-interaction kernels (bench_kernels graph section), the
# gemm.hip shapes incl. the production split-K TN slabs (gemm section), and the wide layers' dual GEMM
# launches at C5's 256 -> 256 on 1M and 300k rows (bench_dual):
# SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_F32, GRBM_GUI_ACTIVE, each program its own run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_mfma_r03
rm -rf $OUT; mkdir -p $OUT
CTR="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE"
WIDE_ROWS=1000000 timeout -s KILL 300 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d $OUT/kern -o run -- \
  python3 tools/bench_kernels.py --only graph,gemm --reps 3 > $OUT/kern.log 2>&1 || { tail -20 $OUT/kern.log; exit 1; }
for rows in 1000000 300000; do
  timeout -s KILL 200 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d $OUT/dual_$rows -o run -- \
    python3 tools/bench_dual.py --rows $rows --din 256 --dout 256 --reps 5 > $OUT/dual_$rows.log 2>&1 \
    || { tail -20 $OUT/dual_$rows.log; exit 1; }
done
python3 tools/pmc_mfma_parse.py $OUT profiles/r03_pmc_mfma.json \
  "tools/bench_kernels.py --only graph,gemm (C2 shapes; gemm.hip at 1M rows incl. the split-K TN slabs); tools/bench_dual.py --rows 1000000/300000 --din 256 --dout 256"
