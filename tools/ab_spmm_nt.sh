set -u
cd "${GRAFT_REPO_ROOT}"
for i in 1 2; do for nt in 0 1; do
  KGAT_SPMM_NT=$nt timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-kg-leg > gpurun_out/ab_nt_${nt}_$i.log 2>&1 || { tail -5 gpurun_out/ab_nt_${nt}_$i.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/ab_nt_${nt}_$i.log') if l.startswith('{')][-1])
print('nt=$nt', round(d['ms_per_step'],4), 'fwd', round(d['spmm']['fwd_avg_ms'],4), 'frontier', round(d['frontier_forward']['ms_per_step'],4))"
done; done
