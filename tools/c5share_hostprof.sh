#!/bin/bash
# Host profile (cProfile) of the C5 rank-share step at a reduced scale: where the host time between a
# step's id all-gather (a device sync) and its first launch goes.  usage: tools/c5share_hostprof.sh SCALE
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=${1:-0.05}
timeout -k 10 1000 python3 -m cProfile -o gpurun_out/c5share_prof.out bench.py --config c5 --scale "$S" --rank-share 8 \
  --steps 3 --warmup 1 --no-cpu-baseline --no-frontier-leg > gpurun_out/c5share_hostprof.log 2>&1 || { tail -20 gpurun_out/c5share_hostprof.log; exit 1; }
tail -1 gpurun_out/c5share_hostprof.log | cut -c1-200
python3 - <<'PY'
import pstats
p = pstats.Stats("gpurun_out/c5share_prof.out")
p.sort_stats("tottime").print_stats(30)
p.sort_stats("cumulative").print_stats("sharded|kernels|model|bench", 40)
PY
