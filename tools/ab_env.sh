#!/bin/bash
# Whole-step A/B of one environment switch: VAR=A_VALUE vs VAR=B_VALUE, interleaved pairs.
# usage: tools/ab_env.sh VAR A_VALUE B_VALUE [pairs]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VAR=$1; AV=$2; BV=$3; N=${4:-2}
for i in $(seq 1 "$N"); do for v in A B; do
  if [ $v = A ]; then val=$AV; else val=$BV; fi
  env "$VAR=$val" timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-kg-leg > gpurun_out/abe_${v}_$i.log 2>&1 || { tail -5 gpurun_out/abe_${v}_$i.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/abe_${v}_$i.log') if l.startswith('{')][-1])
fr=d['frontier_forward']
print('$v', round(d['ms_per_step'],4), 'fwd', round(d['spmm']['fwd_avg_ms'],4), 'frontier', round(fr['ms_per_step'],4), 'bits', fr.get('bit_identical_to_full', {}).get('pass'))"
done; done
