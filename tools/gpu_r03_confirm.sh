#!/bin/bash
# Round-end confirmation on the tree as committed: every GPU test, smoke, the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r03_confirm_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r03_confirm_tests.log | head -30; tail -3 gpurun_out/r03_confirm_tests.log; exit 1; }
tail -1 gpurun_out/r03_confirm_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_confirm_smoke.log 2>&1 || { tail -20 gpurun_out/r03_confirm_smoke.log; exit 1; }
tail -1 gpurun_out/r03_confirm_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/r03_confirm_bench.log 2>&1 || { tail -20 gpurun_out/r03_confirm_bench.log; exit 1; }
tail -1 gpurun_out/r03_confirm_bench.log | cut -c1-400
