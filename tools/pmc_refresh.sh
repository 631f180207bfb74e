#!/bin/bash
# PMC passes over the C2 attention refresh: FETCH_SIZE, WRITE_SIZE and an SQ pass in
# SEPARATE rocprofv3 runs (TCC budget 3 + 2 of 4), kernel-trace only, over bench.py's KG leg (the refresh is
# run 5 times there), then per-launch averages of the row softmax and edge scorer kernels.
# usage: bash tools/pmc_refresh.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05_refresh}
OUT=gpurun_out/pmc_$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  i=$((i + 1))
  timeout -k 10 500 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-frontier-leg > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pmc pass $i ($ctr) rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/p$i.log"; exit $rc; fi
done
python3 - "$OUT" <<'EOF'
import csv, glob, sys
from collections import defaultdict
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if any(s in k for s in ("row_softmax", "edge_score", "slot_sum")):
            vals[k.split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in vals.items():
    print(k)
    for n, v in sorted(c.items()):
        print(f"  {n}: {sum(v) / len(v):.4g} per launch ({len(v)} launches)")
EOF
