#!/bin/bash
# All GPU tests, then the C2 bench twice (short), for a change on the hot path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/gpu_tests.log | head -30; exit $rc; }
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/q.log 2>&1 || { tail -20 gpurun_out/q.log; exit 1; }
  echo "c2: $(tail -1 gpurun_out/q.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["roofline"]["avg_launch_ms"])')"
done
