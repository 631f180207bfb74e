#!/bin/bash
# bi-interaction forward with interleaved-k loads (KGAT_FWD_VARIANT=40) vs the default (8), and the
# forward SpMM with 32x32 row offsets vs the round-start library (ab/libkgat_base.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for rep in 1 2; do
for v in 8 40; do
  KGAT_FWD_VARIANT=$v timeout -k 10 300 python3 tools/bench_kernels.py --only graph --reps 20 > gpurun_out/fwd_v$v.log 2>&1 || { tail -5 gpurun_out/fwd_v$v.log; exit 1; }
  echo "FWD_VARIANT=$v"; grep '"biinter_fwd_' gpurun_out/fwd_v$v.log | cut -c1-150
done
done
for lib in ab/libkgat_base.so problem-recommender-system-using-kgat-in-codeforces_amd/libkgat_hip.so; do
  KGAT_HIP_LIB=$PWD/$lib timeout -k 10 300 python3 tools/bench_kernels.py --only spmm --reps 20 > gpurun_out/spmm_ab.log 2>&1 || { tail -5 gpurun_out/spmm_ab.log; exit 1; }
  echo "$lib"; grep '"spmm_' gpurun_out/spmm_ab.log | cut -c1-150
done
