#!/bin/bash
# A/B: masked-gather edge values loaded for member edges only (variants/libkgat_lazy.so) vs always (base).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for v in base lazy; do
  KGAT_HIP_LIB=variants/libkgat_$v.so timeout -k 10 300 python -u bench.py --steps 40 --no-cpu-baseline --no-parity > gpurun_out/ab_$v.log 2>&1 || { tail -20 gpurun_out/ab_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/ab_$v.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(round(r['ms_per_step'],4), round(r['frontier_forward']['ms_per_step'],4), round(r['spmm']['table_update']['avg_launch_ms'],4), round(r['spmm']['bwd_masked_ms_per_step'],4))")"
done
done
