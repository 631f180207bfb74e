#!/bin/bash
# The wave-specialized fused table update (KGAT_TU_WS variants x blocks per CU) vs the default
# kernel: C2 bench A/B with the table update's kernel time from the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "0 4" "1 4" "2 4" "3 2" "2 2" "0 4"; do
  set -- $cfg
  KGAT_TU_WS=$1 KGAT_TU_WS_BLOCKS=$2 timeout -k 10 300 python -u bench.py --steps 30 --no-cpu-baseline --no-parity \
    --no-kg-leg > gpurun_out/r03_tuws_$1_$2.log 2>&1 || { tail -20 gpurun_out/r03_tuws_$1_$2.log; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/r03_tuws_$1_$2.log').read().strip().splitlines()[-1]); print('TU_WS=$1 blocks/CU=$2', r['ms_per_step'], r['frontier_forward']['ms_per_step'], r['spmm']['table_update']['avg_launch_ms'])"
done
echo done
