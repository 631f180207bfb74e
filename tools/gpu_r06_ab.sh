#!/bin/bash
# Round 6 A/Bs: (1) the row softmax's short rows per wave (KGAT_SOFTMAX_RG 2 vs 4, kernel microbench at C2),
# (2) the small tensors' Adam beside the fused table update (KGAT_SMALL_ADAM_SIDE 1 vs 0, whole C2 steps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do for rg in 2 4; do
  KGAT_SOFTMAX_RG=$rg timeout -k 10 300 python -u tools/bench_kernels.py --only attention,spmm --reps 40 \
    > gpurun_out/sm_ab_${rg}_$i.log 2>&1 || { tail -5 gpurun_out/sm_ab_${rg}_$i.log; exit 1; }
  echo "RG=$rg $(grep row_softmax gpurun_out/sm_ab_${rg}_$i.log)"
done; done
bash tools/ab_env.sh KGAT_SMALL_ADAM_SIDE 1 0 ${PAIRS:-2}
# (3) host cost of the CF step's launches (small graph: host-bound), frontier and full forward
timeout -k 10 200 python -u tools/host_profile.py > gpurun_out/host_cf_frontier.txt 2>&1 && head -3 gpurun_out/host_cf_frontier.txt
timeout -k 10 200 python -u tools/host_profile.py --full > gpurun_out/host_cf_full.txt 2>&1 && head -3 gpurun_out/host_cf_full.txt
