#!/bin/bash
# Lazy CF Adam: parity tests, then the C2 bench (lazy_cf_adam leg) under rocprofv3 --kernel-trace --stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "lazy or captured or frontier or fused or split" > gpurun_out/r04_lazycf_t.log 2>&1 || { tail -30 gpurun_out/r04_lazycf_t.log; exit 1; }
tail -1 gpurun_out/r04_lazycf_t.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_prof_split -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-kg-leg > gpurun_out/r04_prof_split.log 2>&1 || { tail -30 gpurun_out/r04_prof_split.log; exit 1; }
echo done
