#!/bin/bash
# Round 6: the world-8 rehearsals (all ranks on the box's one GPU, gloo) before the driver's 8-GPU run.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=tests/test_gpu_sharded.py
timeout -k 10 1100 python -u -m pytest -m gpu -x -v -p no:cacheprovider --timeout 450 --timeout-method thread \
  "$T::test_dp_exchange_paths_c4_shape[8]" "$T::test_sharded_ranks_one_gpu[8-256:256,128,64-0]" \
  "$T::test_sharded_ranks_one_gpu[8-64:64,32-0]" "$T::test_bench_two_ranks_gloo_rehearsal[replicated-8-c2-0.02]" \
  "$T::test_bench_two_ranks_gloo_rehearsal[sharded-8-c4-0.002]" "$T::test_bench_c5_eight_ranks_gloo_rehearsal" \
  > gpurun_out/r06_w8_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r06_w8_tests.log
exit $rc
