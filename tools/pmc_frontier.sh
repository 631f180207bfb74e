#!/bin/bash
# HBM counters (FETCH_SIZE, WRITE_SIZE: separate passes) of every kernel of the C2 bench incl. its
# frontier-forward leg -> profiles/r02_pmc_frontier_c2.json (the row-set kernels spmm_main<64,5>,
# biinter_fwd<..., true>); profiles/pmc_c2.json (the headline roofline's source) is left as it is.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_frontier
rm -rf $OUT; mkdir -p $OUT
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/$ctr -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity > $OUT/$ctr.log 2>&1
  rc=$?
  echo "pmc $ctr rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/$ctr.log; exit $rc; fi
done
python3 tools/pmc_parse.py $OUT $OUT/r02_pmc_frontier_c2.json "bench.py --steps 5 --warmup 1 (full + frontier legs)" 64 $OUT/FETCH_SIZE.log
