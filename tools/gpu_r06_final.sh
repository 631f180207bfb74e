#!/bin/bash
# Round 6 closing measurements on one GPU.  usage: tools/gpu_r06_final.sh TAG step...
#   tests: the -m gpu suite (-x); smoke: __graft_entry__.smoke(); c2: the driver's default bench line
#   (`python bench.py`: CPU baseline, parity, KG / refresh legs) under a kernel trace, with one full and one
#   frontier step's timelines; c3 / c4: those configs' lines (no CPU baseline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
shift
( while sleep 50; do date +%T >> gpurun_out/${TAG}_heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 450 --timeout-method thread \
        > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_tests.log | head -30; tail -3 gpurun_out/${TAG}_tests.log; exit 1; }
      tail -1 gpurun_out/${TAG}_tests.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
      tail -1 gpurun_out/${TAG}_smoke.log ;;
    c2)
      rm -rf gpurun_out/${TAG}_c2prof
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c2prof -o run --output-format csv -- \
        python3 -u bench.py > gpurun_out/${TAG}_c2_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_c2_bench.log; exit 1; }
      T=$(find gpurun_out/${TAG}_c2prof -name "*kernel_trace.csv" | head -1)
      python3 tools/step_timeline.py "$T" bpr_fwd_kernel 5 > gpurun_out/${TAG}_c2_full_step.txt
      python3 tools/step_timeline.py "$T" bpr_fwd_kernel 30 > gpurun_out/${TAG}_c2_frontier_step.txt
      tail -1 gpurun_out/${TAG}_c2_full_step.txt; tail -1 gpurun_out/${TAG}_c2_frontier_step.txt
      grep "^{" gpurun_out/${TAG}_c2_bench.log | tail -1 | cut -c1-300 ;;
    c2plain)
      timeout -k 10 900 python3 -u bench.py > gpurun_out/${TAG}_c2plain_bench.log 2>&1 \
        || { tail -30 gpurun_out/${TAG}_c2plain_bench.log; exit 1; }
      grep "^{" gpurun_out/${TAG}_c2plain_bench.log | tail -1 | cut -c1-300 ;;
    c3|c4)
      timeout -k 10 900 python3 -u bench.py --config $step --no-cpu-baseline > gpurun_out/${TAG}_${step}_bench.log 2>&1 \
        || { tail -30 gpurun_out/${TAG}_${step}_bench.log; exit 1; }
      grep "^{" gpurun_out/${TAG}_${step}_bench.log | tail -1 | cut -c1-300 ;;
  esac
done
echo done
