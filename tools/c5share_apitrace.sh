#!/bin/bash
# Kernel + HIP API trace of the C5 rank-share step at a reduced scale (where the host gap between a step's
# update and the next step's first copy goes).  usage: tools/c5share_apitrace.sh SCALE
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=${1:-0.1}
rm -rf gpurun_out/c5share_api
timeout -k 10 900 rocprofv3 --kernel-trace --hip-trace -d gpurun_out/c5share_api -o run --output-format csv -- \
  python3 bench.py --config c5 --scale "$S" --rank-share 8 --steps 3 --warmup 1 --no-cpu-baseline --no-frontier-leg \
  > gpurun_out/c5share_api.log 2>&1 || { tail -20 gpurun_out/c5share_api.log; exit 1; }
tail -1 gpurun_out/c5share_api.log | cut -c1-200
ls gpurun_out/c5share_api
