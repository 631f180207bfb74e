#!/bin/bash
# Round 4 measurements on one GPU: the default bench line (C2, with CPU baseline + parity + the KG /
# captured-KG legs), C3 (KGAT d=128 x3 + NFM head), the C5 rehearsal (pipelined row-sharded forward at
# world 1 is a no-op: world 1 runs whole launches), and the rocprof kernel stats of C2 and C3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k nfm > gpurun_out/r04_nfm_tests.log 2>&1 || { tail -30 gpurun_out/r04_nfm_tests.log; exit 1; }
tail -1 gpurun_out/r04_nfm_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/r04_c2_bench.log 2>&1 || { tail -30 gpurun_out/r04_c2_bench.log; exit 1; }
tail -1 gpurun_out/r04_c2_bench.log | cut -c1-600
timeout -k 10 600 python -u bench.py --config c3 > gpurun_out/r04_c3_bench.log 2>&1 || { tail -30 gpurun_out/r04_c3_bench.log; exit 1; }
tail -1 gpurun_out/r04_c3_bench.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_prof_c2 -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-kg-leg --no-frontier-leg > gpurun_out/r04_prof_c2.log 2>&1 || { tail -20 gpurun_out/r04_prof_c2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_prof_c3 -o run --output-format csv -- \
  python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-kg-leg --no-frontier-leg > gpurun_out/r04_prof_c3.log 2>&1 || { tail -20 gpurun_out/r04_prof_c3.log; exit 1; }
echo done
