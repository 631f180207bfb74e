#!/bin/bash
# Round 6: FETCH_SIZE / WRITE_SIZE passes (separate, tools/pmc_bench.sh) over one full-size C5
# rank share -> profiles/pmc_c5_share.json, keyed by the share's rows / entries of A (bench.roofline then
# prices that share's forward SpMM by the counters).  A heartbeat file keeps the host-side graph draw visible.
# usage: bash tools/gpu_r06_pmc_share.sh SHARE_RANK
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
( while sleep 50; do date +%T >> gpurun_out/pmc_share_heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
PMC_NAME=c5_share bash tools/pmc_bench.sh c5 --rank-share 8 --share-rank "${1:-2}" --no-frontier-leg
