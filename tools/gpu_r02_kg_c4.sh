#!/bin/bash
# TransR MFMA forward (tests + fwd timing vs the per-sample kernel) and the C4 step with the
# re-chunked weight-gradient GEMM (tests + bench + rocprof stats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "kg or transr or gemm or wide or d128 or d256 or dense_backward" > gpurun_out/kg_tests.log 2>&1; rc=$?
tail -2 gpurun_out/kg_tests.log
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/kg_tests.log | head -30; exit $rc; }
for d in 64 128 256; do for sk in "" "--skew"; do
  timeout -k 10 120 python -u tools/bench_kg.py --dim $d $sk >> gpurun_out/kg_bench.log 2>&1 || { tail -5 gpurun_out/kg_bench.log; exit 1; }
  KGAT_TRANSR_VALU=1 timeout -k 10 120 python -u tools/bench_kg.py --dim $d $sk | sed 's/"transr"/"transr_valu"/' >> gpurun_out/kg_bench.log 2>&1 || { tail -5 gpurun_out/kg_bench.log; exit 1; }
done; done
cat gpurun_out/kg_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
  python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/bench_c4.log 2>&1 || { tail -20 gpurun_out/bench_c4.log; exit 1; }
timeout -k 10 400 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/bench_c4_noprof.log 2>&1 || { tail -20 gpurun_out/bench_c4_noprof.log; exit 1; }
tail -1 gpurun_out/bench_c4_noprof.log | cut -c1-300
