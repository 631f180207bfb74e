#!/bin/bash
# MFMA utilisation of the MFMA-bound kernels (bi-interaction fwd/bwd, edge scorer, NFM) at C2
# shapes: SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_F32 and GRBM_GUI_ACTIVE in one
# --pmc pass (SQ 2 of 8 slots, GRBM 1 of 2), kernel-trace only; parsed by tools/pmc_mfma_parse.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_mfma
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $OUT/run -o run -- \
  python3 tools/bench_kernels.py --only graph,attention,nfm --reps 3 > $OUT/run.log 2>&1
rc=$?
echo "pmc rc=$rc"
if [ $rc -ne 0 ]; then tail -20 $OUT/run.log; exit $rc; fi
python3 tools/pmc_mfma_parse.py $OUT profiles/pmc_mfma_c2.json
