#!/bin/bash
# C3 under a kernel trace (kernel stats + one full and one frontier step timeline).  usage: tools/gpu_r06_c3prof.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06c3}
rm -rf gpurun_out/${TAG}_prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
  python3 -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-kg-leg \
  > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
T=$(find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py "$T" bpr_fwd_kernel 5 > gpurun_out/${TAG}_full_step.txt
python3 tools/step_timeline.py "$T" bpr_fwd_kernel 18 > gpurun_out/${TAG}_frontier_step.txt
tail -1 gpurun_out/${TAG}_full_step.txt; tail -1 gpurun_out/${TAG}_frontier_step.txt
grep "^{" gpurun_out/${TAG}_bench.log | tail -1 | cut -c1-200
