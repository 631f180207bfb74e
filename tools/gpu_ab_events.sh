#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for ev in 1 4 1000; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-parity --event-every $ev > gpurun_out/ev.log 2>&1 || { tail -20 gpurun_out/ev.log; exit 1; }
  echo "event-every $ev: $(tail -1 gpurun_out/ev.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["roofline"]["avg_launch_ms"], r["spmm"]["event_steps"])')"
done
done
