#!/bin/bash
# early zero rows with the step on a high-priority stream (side stream at the default priority)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "0 0" "1 -1" "0 -1" "1 -1"; do
  set -- $cfg
  KGAT_TU_EARLY=$1 KGAT_MAIN_PRIO=$2 timeout -k 10 400 python -u bench.py --steps 30 --no-cpu-baseline --no-parity --no-kg-leg \
    > gpurun_out/prio.log 2>&1 || { tail -20 gpurun_out/prio.log; exit 1; }
  python3 -c "
import json; r=json.loads(open('gpurun_out/prio.log').read().strip().splitlines()[-1])
print('early=$1 mainprio=$2', 'full %.4f' % r['ms_per_step'], 'frontier %.4f' % r['frontier_forward']['ms_per_step'], 'tu(part1) %.4f' % r['spmm']['table_update']['avg_launch_ms'], 'bitid', r['frontier_forward']['bit_identical_to_full']['pass'])"
done
