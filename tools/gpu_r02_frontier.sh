#!/bin/bash
# Frontier-restricted forward: bit-identity tests, the new ABI entries, then the C2 bench with its frontier leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "frontier_forward or fused_table_update or driver or test_cf or hop_chain" > gpurun_out/frontier_tests.log 2>&1; rc=$?
tail -3 gpurun_out/frontier_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/frontier_tests.log | head -40; exit $rc; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-parity > gpurun_out/frontier_bench.log 2>&1 || { tail -30 gpurun_out/frontier_bench.log; exit 1; }
tail -1 gpurun_out/frontier_bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms_per_step'], r['frontier_forward'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fr -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/prof_fr.log 2>&1 || { tail -20 gpurun_out/prof_fr.log; exit 1; }
echo done
