#!/bin/bash
# Round 5: one rank's full-size C5 share on one GPU -- rank 0 of 8's rows of A and A^T
# (graph.HashedCKG, N = 50M, 500M triples, d = 256, layers [256, 128, 64]), the full [N, d] gathered layer
# buffers filled locally (bench.ShareComm), under a kernel trace.  A heartbeat file keeps the long host-side
# graph generation visible as progress.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 50; do date +%T >> gpurun_out/r05_c5share_heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
SCALE=${1:-1}
rm -rf gpurun_out/r05_c5share_trace
timeout -k 10 1080 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_c5share_trace -o run --output-format csv -- \
  python3 -u bench.py --config c5 --scale "$SCALE" --rank-share 8 --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r05_c5share.log 2>&1 || { tail -30 gpurun_out/r05_c5share.log; exit 1; }
grep -v "^{" gpurun_out/r05_c5share.log | tail -8
tail -1 gpurun_out/r05_c5share.log | cut -c1-600
echo done
