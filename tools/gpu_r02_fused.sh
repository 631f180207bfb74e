#!/bin/bash
# Fused layer-0 product + table Adam: parity tests, then C2 / C4 A/B (fused vs --no-fused-update).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "fused_table_update or hop_chain or dp_ or replicated or driver or smoke or cf_train_steps" > gpurun_out/fused_tests.log 2>&1; rc=$?
tail -3 gpurun_out/fused_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/fused_tests.log | head -30; exit $rc; }
for mode in "" "--no-fused-update" ""; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-parity $mode > gpurun_out/bench_c2_ab.log 2>&1 || { tail -20 gpurun_out/bench_c2_ab.log; exit 1; }
  echo "c2 [$mode]: $(tail -1 gpurun_out/bench_c2_ab.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["spmm"]["bwd_masked_ms_per_step"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2f -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/bench_c2_prof.log 2>&1 || { tail -20 gpurun_out/bench_c2_prof.log; exit 1; }
for mode in "" "--no-fused-update"; do
  timeout -k 10 400 python -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-parity $mode > gpurun_out/bench_c4_ab.log 2>&1 || { tail -20 gpurun_out/bench_c4_ab.log; exit 1; }
  echo "c4 [$mode]: $(tail -1 gpurun_out/bench_c4_ab.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["spmm"]["bwd_masked_ms_per_step"])')"
done
