#!/bin/bash
# Kernel-time A/B of library builds (abx/lib_*.so) on the C2 bench: rocprofv3 kernel stats per build,
# interleaved twice; prints the bi-interaction forward and the step's top kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for V in "$@"; do
D=gpurun_out/biab_${V}_$rep
KGAT_HIP_LIB=$PWD/abx/lib_$V.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-parity --no-kg-leg --steps 10 --warmup 3 > $D.log 2>&1 || { tail -20 $D.log; exit 1; }
python3 - "$D" "$V" "$rep" <<'PY'
import csv, glob, json, sys
D, V, rep = sys.argv[1:]
f = glob.glob(f"{D}/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
line = [l for l in open(D + ".log") if l.startswith('{"metric"')][-1]
d = json.loads(line)
print(V, rep, "full %.4f" % d["ms_per_step"], "frontier %.4f" % d["frontier_forward"]["ms_per_step"])
for r in rows:
    if "biinter" in r["Name"] or "spmm_main" in r["Name"]:
        print("   %-60.60s calls %5s avg %8.1f us" % (r["Name"], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
done
