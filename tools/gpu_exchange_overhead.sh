#!/bin/bash
# The N-rank exchange paths: DP / RCCL tests, then the exchange's overhead at world 1 (RCCL, no data
# between GPUs): C2 step time plain vs --exchange-at-1 (replicated / sharded), and a kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "dp_ or rccl or rehearsal or fused_table or sharded_world" > gpurun_out/xo_tests.log 2>&1; rc=$?
tail -2 gpurun_out/xo_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/xo_tests.log | head -30; tail -30 gpurun_out/dp_world2.log; exit $rc; }
for mode in "" "--exchange-at-1 --dp replicated" "--exchange-at-1 --dp sharded"; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-parity $mode > gpurun_out/xo.log 2>&1 || { tail -20 gpurun_out/xo.log; exit 1; }
  echo "c2 [$mode]: $(tail -1 gpurun_out/xo.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r.get("dp_table_exchange_steps"))')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_xo -o run -- \
  python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --exchange-at-1 --dp replicated > gpurun_out/prof_xo.log 2>&1 || { tail -20 gpurun_out/prof_xo.log; exit 1; }
