#!/bin/bash
# Round 4 confirmation on one GPU: the whole GPU suite, smoke(), the default bench line (C2, CPU baseline +
# parity + KG legs), the C3 line, and the rocprof kernel stats of the C2 CF step (full + frontier legs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/r04_final_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r04_final_tests.log | head -30; tail -3 gpurun_out/r04_final_tests.log; exit 1; }
tail -1 gpurun_out/r04_final_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_final_smoke.log 2>&1 || { tail -20 gpurun_out/r04_final_smoke.log; exit 1; }
tail -2 gpurun_out/r04_final_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r04_final_c2_bench.log 2>&1 || { tail -30 gpurun_out/r04_final_c2_bench.log; exit 1; }
tail -1 gpurun_out/r04_final_c2_bench.log | cut -c1-400
timeout -k 10 600 python -u bench.py --config c3 > gpurun_out/r04_final_c3_bench.log 2>&1 || { tail -30 gpurun_out/r04_final_c3_bench.log; exit 1; }
tail -1 gpurun_out/r04_final_c3_bench.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_final_prof_c2 -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-kg-leg > gpurun_out/r04_final_prof_c2.log 2>&1 || { tail -20 gpurun_out/r04_final_prof_c2.log; exit 1; }
echo done
