set -e
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in hop batch; do
  rm -rf gpurun_out/tp_$s
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tp_$s -o run --output-format csv -- python3 -u tools/tiles_probe.py $s > gpurun_out/tp_$s.log 2>&1
  f=$(find gpurun_out/tp_$s -name "*kernel_stats.csv" | head -1)
  grep -E "biinter_fwd_set|biinter_fwd_kernel" "$f" | cut -d, -f1-8 | sed "s/^/$s: /"
done
