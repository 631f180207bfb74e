#!/bin/bash
# Whole-step A/B of two library builds (gpurun_ab/libA.so, gpurun_ab/libB.so), interleaved pairs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do for v in A B; do
  KGAT_HIP_LIB=$PWD/gpurun_ab/lib$v.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-kg-leg > gpurun_out/ab_${v}_$i.log 2>&1 || { tail -5 gpurun_out/ab_${v}_$i.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/ab_${v}_$i.log') if l.startswith('{')][-1])
print('$v', round(d['ms_per_step'],4), 'fwd', round(d['spmm']['fwd_avg_ms'],4), 'frontier', round(d['frontier_forward']['ms_per_step'],4))"
done; done
