#!/bin/bash
# HBM traffic per kernel of the bench step from PMC counters: FETCH_SIZE and WRITE_SIZE in SEPARATE
# rocprofv3 passes (TCC slot budget: 3 + 2 of 4), kernel-trace only, over `bench.py --config CFG`
# itself (every kernel of the timed step, this exact build), then tools/pmc_parse.py ->
# profiles/pmc_CFG.json.   usage: bash tools/pmc_bench.sh c2 [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
cfg=${1:-c2}; shift || true
NAME=${PMC_NAME:-$cfg}  # the profiles/pmc_NAME.json the counters go to (c5_share for a rank share)
OUT=gpurun_out/pmc_$NAME
rm -rf $OUT; mkdir -p $OUT
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/$ctr -o run -- \
    python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-parity "$@" > $OUT/$ctr.log 2>&1
  rc=$?
  echo "pmc $ctr rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/$ctr.log; exit $rc; fi
done
case $cfg in c3|c4) d0=128;; c5) d0=256;; *) d0=64;; esac
python3 tools/pmc_parse.py $OUT profiles/pmc_$NAME.json "bench.py --config $cfg --steps 5 --warmup 1 $*" $d0 $OUT/FETCH_SIZE.log && cp profiles/pmc_$NAME.json $OUT/
