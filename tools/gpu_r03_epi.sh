#!/bin/bash
# biinter_fwd epilogue-weight probe: the product kernel timed with dropout on / off and with / without the
# saved-state stores, interleaved twice on one box (tools/ab_fwd.py AB_P / AB_STATE).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AB_SHAPES=64x64_n1000000,64x32_n1000000,128x64_n1000000
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "0.1 1" "0 1" "0 0"; do
    set -- $cfg
    AB_P=$1 AB_STATE=$2 timeout -k 10 300 python3 tools/ab_fwd.py gpurun_out/epi_${1}_${2}_$r.json > gpurun_out/epi_${1}_${2}_$r.log 2>&1 || { tail -5 gpurun_out/epi_${1}_${2}_$r.log; exit 1; }
    echo "p=$1 state=$2 round=$r"; grep -E "^[0-9]+x" gpurun_out/epi_${1}_${2}_$r.log
  done
done
