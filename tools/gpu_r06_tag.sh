#!/bin/bash
# Round 6: the id-check tests (tagged TRAIN_CF completion) then the plain C2 bench line and a short C2
# kernel trace (cf_begin's duration).   usage: bash tools/gpu_r06_tag.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06_tag}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "tagged or out_of_range or device_id_error or frontier_forward_bit or fused_table or alternating or dp_ or captured" \
  > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/${TAG}_tests.log | head -20; tail -3 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_c2.log 2>&1 || { tail -20 gpurun_out/${TAG}_c2.log; exit 1; }
grep "^{" gpurun_out/${TAG}_c2.log | tail -1 | cut -c1-200
rm -rf gpurun_out/${TAG}_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
  python3 -u bench.py --no-cpu-baseline --no-parity --steps 10 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
grep -h "cf_begin" gpurun_out/${TAG}_prof/run_kernel_stats.csv | cut -c1-200
echo done
