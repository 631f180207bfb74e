#!/bin/bash
# A/B of the row-set forward SpMM's gathers in flight (variants/libkgat_u{4,8,16}.so): C2 frontier-leg step time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for v in u4 u8 u16; do
  KGAT_HIP_LIB=variants/libkgat_$v.so timeout -k 10 300 python -u bench.py --steps 30 --no-cpu-baseline --no-parity > gpurun_out/ab_$v.log 2>&1 || { tail -20 gpurun_out/ab_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/ab_$v.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(round(r['ms_per_step'],4), round(r['frontier_forward']['ms_per_step'],4))")"
done
done
