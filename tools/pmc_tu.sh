#!/bin/bash
# Fused table update at C2 (tools/bench_tu.py): plain timing of each library variant, then SQ counter
# passes over the default kernel and the dense Adam beside it.  Args: variant env assignments to time,
# e.g.  bash tools/pmc_tu.sh "KGAT_TU_VARIANT=0" "KGAT_TU_VARIANT=1"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
OUT=gpurun_out/pmc_tu
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 python3 tools/bench_tu.py --tag default > $OUT/default.log 2>&1 || { tail -20 $OUT/default.log; exit 1; }
tail -1 $OUT/default.log
for v in "$@"; do
  env $v timeout -k 10 200 python3 tools/bench_tu.py --tag "$v" > $OUT/v.log 2>&1 || { tail -20 $OUT/v.log; exit 1; }
  tail -1 $OUT/v.log
done
[ -n "${PMC_TU:-}" ] || exit 0
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
cd /tmp
for p in 1 2; do
  eval C=\$P$p
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/$OUT/p$p -o run -- \
    python3 $R/tools/bench_tu.py --reps 5 > $R/$OUT/p$p.log 2>&1 || { echo "pass $p failed"; tail -5 $R/$OUT/p$p.log; }
done
python3 $R/tools/pmc_dump.py $R/$OUT "<64, 4>"
python3 $R/tools/pmc_dump.py $R/$OUT adam_multi
