#!/bin/bash
# Lazy CF Adam: parity tests (list walk and per-row stamp test), the C2 bench's lazy_cf_adam leg with
# both, the frontier step's host profile with and without lazy, and the NFM big-LDS A/B at C3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "lazy or captured or frontier or fused or nfm" > gpurun_out/r04_lazycf_t.log 2>&1 || { tail -30 gpurun_out/r04_lazycf_t.log; exit 1; }
tail -1 gpurun_out/r04_lazycf_t.log
KGAT_LAZY_LIST=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "lazy_cf" > gpurun_out/r04_lazycf_t0.log 2>&1 || { tail -30 gpurun_out/r04_lazycf_t0.log; exit 1; }
tail -1 gpurun_out/r04_lazycf_t0.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-parity > gpurun_out/r04_lazycf_bench.log 2>&1 || { tail -30 gpurun_out/r04_lazycf_bench.log; exit 1; }
echo c2 ok
KGAT_LAZY_LIST=0 timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-parity --no-kg-leg > gpurun_out/r04_lazycf_bench0.log 2>&1 || { tail -30 gpurun_out/r04_lazycf_bench0.log; exit 1; }
echo c2 stamp-test ok
timeout -k 10 300 python -u tools/host_profile.py --lazy-cf > gpurun_out/r04_hp_lazycf.log 2>&1 || { tail -30 gpurun_out/r04_hp_lazycf.log; exit 1; }
head -3 gpurun_out/r04_hp_lazycf.log
timeout -k 10 300 python -u tools/host_profile.py > gpurun_out/r04_hp_frontier.log 2>&1 || { tail -30 gpurun_out/r04_hp_frontier.log; exit 1; }
head -3 gpurun_out/r04_hp_frontier.log
timeout -k 10 600 python -u bench.py --config c3 --no-cpu-baseline --no-parity --no-kg-leg > gpurun_out/r04_c3_nfm_a.log 2>&1 || { tail -30 gpurun_out/r04_c3_nfm_a.log; exit 1; }
KGAT_NFM_WLDS_BIG=1 timeout -k 10 600 python -u bench.py --config c3 --no-cpu-baseline --no-parity --no-kg-leg > gpurun_out/r04_c3_nfm_b.log 2>&1 || { tail -30 gpurun_out/r04_c3_nfm_b.log; exit 1; }
echo done
