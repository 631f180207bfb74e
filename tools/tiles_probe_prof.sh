#!/bin/bash
# The row-set forward probe (tools/tiles_probe.py) under a kernel trace, one set per run: the per-kernel
# durations are the measurement (the probe's own event timings of small sets are host-bound).
set -e
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in hop batch; do
  rm -rf gpurun_out/tp_$s
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tp_$s -o run --output-format csv -- \
    python3 -u tools/tiles_probe.py $s > gpurun_out/tp_$s.log 2>&1
  f=$(find gpurun_out/tp_$s -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$s" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "biinter_fwd" in r["Name"]:
        print(sys.argv[2], r["Name"][:60], r["Calls"], "avg us", round(float(r["AverageNs"]) / 1e3, 1))
PY
done
