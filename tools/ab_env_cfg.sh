#!/bin/bash
# A/B of one environment switch on another bench config: VAR=A vs VAR=B, interleaved pairs.
# usage: tools/ab_env_cfg.sh CONFIG VAR A_VALUE B_VALUE [pairs]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=$1; VAR=$2; AV=$3; BV=$4; N=${5:-2}
for i in $(seq 1 "$N"); do for v in A B; do
  if [ $v = A ]; then val=$AV; else val=$BV; fi
  env "$VAR=$val" timeout -k 10 400 python -u bench.py --config "$CFG" --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-kg-leg > gpurun_out/abc_${v}_$i.log 2>&1 || { tail -5 gpurun_out/abc_${v}_$i.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/abc_${v}_$i.log') if l.startswith('{')][-1])
print('$v', round(d['ms_per_step'],4), 'fwd', round(d['spmm']['fwd_avg_ms'],4), 'frontier', round(d.get('frontier_forward',{}).get('ms_per_step',0),4))"
done; done
