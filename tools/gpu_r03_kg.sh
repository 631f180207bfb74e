#!/bin/bash
# KG step: the KG / lazy tests, host profiles of the fused and lazy KG steps, and the C4 bench's KG legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "lazy or kg or id_error or frontier_forward_bit" > gpurun_out/r03_kg_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r03_kg_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/r03_kg_tests.log | head -30; exit $rc; }
for a in "--kg" "--kg --lazy"; do
  timeout -k 10 300 python3 tools/host_profile.py $a > "gpurun_out/hp$(echo $a | tr -d ' -').log" 2>&1 || exit 1
  grep "kg:" "gpurun_out/hp$(echo $a | tr -d ' -').log"
done
timeout -k 10 900 python -u bench.py --config c4 --steps 4 --warmup 2 --no-cpu-baseline --no-parity --no-frontier-leg \
  > gpurun_out/r03_c4_kg.log 2>&1 || { tail -20 gpurun_out/r03_c4_kg.log; exit 1; }
tail -1 gpurun_out/r03_c4_kg.log | cut -c1-200
