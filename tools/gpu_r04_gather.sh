#!/bin/bash
# Masked gather with LDS-compacted hits: the GPU parity suite, then the C2 bench under rocprofv3 --stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04_gather_t.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r04_gather_t.log | head -20; tail -3 gpurun_out/r04_gather_t.log; exit 1; }
tail -1 gpurun_out/r04_gather_t.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_prof_gather -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-kg-leg > gpurun_out/r04_prof_gather.log 2>&1 || { tail -30 gpurun_out/r04_prof_gather.log; exit 1; }
echo done
