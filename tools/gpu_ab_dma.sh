#!/bin/bash
# DMA-fed bi-interaction forward: parity tests, then kernel A/B (8 / 12 / 4 waves, register-loaded) and the C2 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "biinter or cf_ or golden or hop or smoke or parity" > gpurun_out/dma_tests.log 2>&1; rc=$?
tail -2 gpurun_out/dma_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/dma_tests.log | head -30; exit $rc; }
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u tools/bench_kernels.py --only graph --reps 20 > gpurun_out/abdma_$name.log 2>&1 || { tail -5 gpurun_out/abdma_$name.log; exit 1; }
  echo "$name: $(grep biinter_fwd_saved gpurun_out/abdma_$name.log | tr '\n' ' ')"
}
run dma8 KGAT_X=1
run dma12 KGAT_HIP_LIB=variants/libkgat_w12.so
run dma4 KGAT_HIP_LIB=variants/libkgat_w4.so
run regs KGAT_FWD_VARIANT=24
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/abdma_bench.log 2>&1 || { tail -5 gpurun_out/abdma_bench.log; exit 1; }
echo "bench dma8 $(tail -1 gpurun_out/abdma_bench.log | grep -o '"ms_per_step": [0-9.]*')"
