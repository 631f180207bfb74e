#!/bin/bash
# A/B the bi-interaction forward variants (KGAT_FWD_VARIANT) on the C2 microbench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 0 4 8 12 14; do
  KGAT_FWD_VARIANT=$v timeout -k 10 200 python tools/bench_kernels.py --only fused > gpurun_out/fwdv_$v.log 2>&1 || exit 1
  echo "variant=$v $(grep 'spmm+biinter' gpurun_out/fwdv_$v.log | tr '\n' ' ')"
done
