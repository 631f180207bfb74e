#!/bin/bash
# HBM traffic of the dominant kernel (forward SpMM, d=64, C2 graph) from PMC
# counters: FETCH_SIZE and WRITE_SIZE in SEPARATE rocprofv3 passes (TCC slot
# budget), kernel-trace only, then tools/pmc_parse.py -> profiles/pmc_c2.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/$ctr -o run -- \
    python3 tools/bench_kernels.py --only spmm --reps 5 > $OUT/$ctr.log 2>&1
  rc=$?
  echo "pmc $ctr rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/$ctr.log; exit $rc; fi
done
python3 tools/pmc_parse.py $OUT profiles/pmc_c2.json && cp profiles/pmc_c2.json $OUT/
