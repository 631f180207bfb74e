#!/bin/bash
# Round 3: the C5 path's new pieces -- hop backward and frontier forward of the row-sharded model,
# the dual-GEMM wide bi-interaction -- tested (sharded worlds 1/2/4 incl. the frontier check, wide
# bi-interaction parity, dual vs separate bit identity), then the C5 rehearsal (2 % scale, world 1,
# with its frontier leg and oracle parity) under rocprofv3 --stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_gemm.py tests/test_gpu_sharded.py \
  -k "dual_gemm or gemm_rows or mark_rows or biinter_wide or bwd_rows or gemm or sharded or rehearsal or 256 or L3" \
  > gpurun_out/r03_c5opt_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r03_c5opt_tests.log
grep -h "bit-identical" gpurun_out/sharded_world*.log | head -12
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/r03_c5opt_tests.log | head -40; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5f -o run --output-format csv -- \
  python3 bench.py --config c5 --scale 0.02 --steps 8 --warmup 2 > gpurun_out/r03_c5f.log 2>&1 || { tail -20 gpurun_out/r03_c5f.log; exit 1; }
tail -1 gpurun_out/r03_c5f.log | cut -c1-300
