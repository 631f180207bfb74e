#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for sc in 0.01 1; do
for mode in "" "--exchange-at-1 --dp replicated"; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-parity --scale $sc $mode > gpurun_out/xo.log 2>&1 || { tail -20 gpurun_out/xo.log; exit 1; }
  echo "scale $sc [$mode]: $(tail -1 gpurun_out/xo.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["host_launch_ms_per_step"])')"
done
done
