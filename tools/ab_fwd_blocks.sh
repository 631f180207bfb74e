cd $GRAFT_REPO_ROOT
for b in 0 2 4; do
  KGAT_FWD_BLOCKS=$b timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$b.log 2>&1 || exit 1
  echo "blocks=$b $(tail -1 gpurun_out/ab_$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['spmm']['fwd_avg_ms'], d['spmm']['fwd_launches'])")"
done
