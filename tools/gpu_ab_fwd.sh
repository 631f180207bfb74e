#!/bin/bash
# A/B of the bi-interaction forward launch variants (KGAT_FWD_VARIANT) at C2 shapes, then the C2 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 8 12 0 4 10 14; do
  KGAT_FWD_VARIANT=$v timeout -k 10 300 python -u tools/bench_kernels.py --only graph --reps 20 > gpurun_out/abfwd_$v.log 2>&1 || { tail -5 gpurun_out/abfwd_$v.log; exit 1; }
  echo "variant $v: $(grep biinter_fwd_saved gpurun_out/abfwd_$v.log | tr '\n' ' ')"
done
for v in 8 12; do
  KGAT_FWD_VARIANT=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/abfwd_bench_$v.log 2>&1 || { tail -5 gpurun_out/abfwd_bench_$v.log; exit 1; }
  echo "bench $v $(tail -1 gpurun_out/abfwd_bench_$v.log | grep -o '"ms_per_step": [0-9.]*')"
done
