#!/bin/bash
# Whole-step A/B of an environment switch: bash tools/ab_bench_env.sh VAR v1 v2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
var=$1; shift
for v in "$@"; do
  env "$var=$v" timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || exit 1
  echo "$var=$v $(tail -1 gpurun_out/ab_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), round(d['spmm']['fwd_avg_ms'],4))")"
done
