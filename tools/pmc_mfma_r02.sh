#!/bin/bash
# Round-2 MFMA utilisation pass: the C2 MFMA kernels + C4's wide layers + the library GEMM
# (bench_kernels), and TransR's W_r.e MFMA forward at d = 64 / 256 (bench_kg, B = 512 and 8192):
# SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_F32, GRBM_GUI_ACTIVE, each program its own run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_mfma_r02
rm -rf $OUT; mkdir -p $OUT
CTR="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d $OUT/kern -o run -- \
  python3 tools/bench_kernels.py --only graph,attention,nfm,wide,gemm --reps 3 > $OUT/kern.log 2>&1 || { tail -20 $OUT/kern.log; exit 1; }
for d in 64 256; do
  for b in 512 8192; do
    timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d $OUT/kg_${d}_$b -o run -- \
      python3 tools/bench_kg.py --dim $d --batch $b --reps 5 > $OUT/kg_${d}_$b.log 2>&1 || { tail -20 $OUT/kg_${d}_$b.log; exit 1; }
  done
done
python3 tools/pmc_mfma_parse.py $OUT profiles/r02_pmc_mfma.json \
  "tools/bench_kernels.py --only graph,attention,nfm,wide,gemm (C2 shapes, C4 wide layers); tools/bench_kg.py --dim 64/256 --batch 512/8192"
