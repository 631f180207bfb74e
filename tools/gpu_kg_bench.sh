#!/bin/bash
# TransR KG step: parity tests, kernel microbench (uniform / skewed relations), one profiled train-sm epoch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "kg_" --timeout 120 --timeout-method thread > gpurun_out/gpu_kg.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_kg.log
[ $rc -ne 0 ] && exit $rc
for a in "" "--skew" "--dim 256" "--batch 64"; do
  timeout -k 10 120 python tools/bench_kg.py $a > gpurun_out/kg_bench.log 2>&1 || { tail -20 gpurun_out/kg_bench.log; exit 1; }
  grep kernel gpurun_out/kg_bench.log
done
rm -rf gpurun_out/prof_sm gpurun_out/result_sm3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sm -o run --output-format csv -- python tools/kgat_main.py --sm --epochs 1 --result-dir gpurun_out/result_sm3 > gpurun_out/prof_sm.log 2>&1 || { tail -20 gpurun_out/prof_sm.log; exit 1; }
grep epoch gpurun_out/prof_sm.log
