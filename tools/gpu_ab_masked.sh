#!/bin/bash
# A/B of the layer-0 masked A^T product variants (variants/libkgat_*.so) + C4 step with the split-K change.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "hop_chain or gemm or wide or masked or dense_backward or c4 or d128 or d256" > gpurun_out/ab_tests.log 2>&1; rc=$?
tail -3 gpurun_out/ab_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/ab_tests.log | head -30; exit $rc; }
for v in u0 u4 u8; do
  KGAT_HIP_LIB=variants/libkgat_$v.so timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/ab_bench_$v.log 2>&1 || { tail -5 gpurun_out/ab_bench_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/ab_bench_$v.log | grep -o '"ms_per_step": [0-9.]*') $(tail -1 gpurun_out/ab_bench_$v.log | grep -o '"bwd_masked_ms_per_step": [0-9.]*')"
done
timeout -k 10 400 python -u bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/ab_c4.log 2>&1 || { tail -5 gpurun_out/ab_c4.log; exit 1; }
echo "c4 $(tail -1 gpurun_out/ab_c4.log | grep -o '"ms_per_step": [0-9.]*') $(tail -1 gpurun_out/ab_c4.log | grep -o '"bwd_masked_ms_per_step": [0-9.]*')"
