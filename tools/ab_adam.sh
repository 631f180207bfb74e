#!/bin/bash
# A/B the multi-tensor Adam variants (KGAT_ADAM_VARIANT) on the C2 table (64M parameters).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 0 1 2; do
  KGAT_ADAM_VARIANT=$v timeout -k 10 200 python tools/bench_kernels.py --only graph > gpurun_out/adam_$v.log 2>&1 || exit 1
  grep adam_multi gpurun_out/adam_$v.log
done
