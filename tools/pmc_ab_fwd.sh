#!/bin/bash
# Counter passes over the bi-interaction forward (64->64, 1M rows), register path vs LDS-DMA path.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcfwd
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
export AB_SHAPES=64x64_n1000000
for v in 8 24; do
  for p in 1 2; do
    eval C=\$P$p
    KGAT_FWD_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmcfwd/v${v}_p$p -o run -- python3 $R/tools/ab_fwd.py /tmp/x.json > $R/gpurun_out/pmcfwd/v${v}_p$p.log 2>&1 || exit $?
  done
done
python3 $R/tools/pmc_dump.py $R/gpurun_out/pmcfwd biinter_fwd
