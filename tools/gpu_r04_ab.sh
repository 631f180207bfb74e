#!/bin/bash
# Interleaved A/B of two library builds (abx/lib_*.so) on the C2 bench step (table-update launch time).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for V in "$@"; do
KGAT_HIP_LIB=$PWD/abx/lib_$V.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity --no-kg-leg > gpurun_out/r04_ab_${V}_$rep.log 2>&1 || { tail -20 gpurun_out/r04_ab_${V}_$rep.log; exit 1; }
python3 - "$V" "$rep" <<'PY'
import json, sys
V, rep = sys.argv[1], sys.argv[2]
line = [l for l in open(f"gpurun_out/r04_ab_{V}_{rep}.log") if l.startswith('{"metric"')][-1]
d = json.loads(line)
print(V, rep, "full %.4f" % d["ms_per_step"], "frontier %.4f" % d["frontier_forward"]["ms_per_step"],
      "tu %.4f" % d["spmm"]["table_update"]["avg_launch_ms"], "fwd %.4f" % d["spmm"]["fwd_avg_ms"])
PY
done
done
