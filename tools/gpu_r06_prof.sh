#!/bin/bash
# Round 6: one C2 bench under a kernel trace (per-step timelines of the full and the frontier step, kernel
# stats) + the row softmax's kernels under RG = 2 / 4 (KGAT_SOFTMAX_RG) at C2.  usage: tools/gpu_r06_prof.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06prof}
rm -rf gpurun_out/${TAG}_prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-kg-leg \
  > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
T=$(find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py "$T" bpr_fwd_kernel 5 > gpurun_out/${TAG}_full_step.txt
python3 tools/step_timeline.py "$T" bpr_fwd_kernel -6 > gpurun_out/${TAG}_frontier_step.txt
tail -1 gpurun_out/${TAG}_full_step.txt
tail -1 gpurun_out/${TAG}_frontier_step.txt
for rg in 2 4; do
  rm -rf gpurun_out/${TAG}_sm$rg
  KGAT_SOFTMAX_RG=$rg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_sm$rg -o run \
    --output-format csv -- python3 tools/bench_kernels.py --only attention,spmm --reps 20 \
    > gpurun_out/${TAG}_sm$rg.log 2>&1 || { tail -5 gpurun_out/${TAG}_sm$rg.log; exit 1; }
  S=$(find gpurun_out/${TAG}_sm$rg -name "*kernel_stats.csv" | head -1)
  echo "RG=$rg"; grep -i "softmax\|seg_write" "$S" | cut -d, -f1-5
done
