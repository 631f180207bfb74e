#!/bin/bash
# Round 6: full-size C5 rank shares on one GPU -- by default rank 0 (the most edges) and the
# rank with the most rows, one drawn graph (graph.HashedCKG, N = 50M, 500M triples, d = 256, [256, 128, 64]),
# under a kernel trace.  usage: bash tools/gpu_r06_c5share.sh TAG "SHARE_RANKS" [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06_c5share}; RANKS=${2:-0,maxrows}; shift 2 || true
( while sleep 50; do date +%T >> gpurun_out/${TAG}_heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
rm -rf gpurun_out/${TAG}_trace
timeout -k 10 1100 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o run --output-format csv -- \
  python3 -u bench.py --config c5 --rank-share 8 --share-rank "$RANKS" --steps 3 --warmup 1 --no-cpu-baseline "$@" \
  > gpurun_out/${TAG}.log 2>&1 || { tail -30 gpurun_out/${TAG}.log; exit 1; }
grep -v "^{" gpurun_out/${TAG}.log | grep -v "^[WE]2026" | tail -12
tail -1 gpurun_out/${TAG}.log | cut -c1-400
echo done
