set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -6 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
rm -rf gpurun_out/prof_sm gpurun_out/result_sm3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sm -o run --output-format csv -- python tools/kgat_main.py --sm --epochs 1 --result-dir gpurun_out/result_sm3 > gpurun_out/prof_sm.log 2>&1 || { tail -20 gpurun_out/prof_sm.log; exit 1; }
grep epoch gpurun_out/prof_sm.log
head -6 gpurun_out/prof_sm/run_kernel_stats.csv | cut -c1-160
