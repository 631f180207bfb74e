#!/bin/bash
# A/B of two library builds (ab/libkgat_base.so vs the in-tree libkgat_hip.so) on the C2 bench,
# interleaved base / new / base / new.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
NEW=problem-recommender-system-using-kgat-in-codeforces_amd/libkgat_hip.so
for rep in 1 2; do
  for lib in ab/libkgat_base.so $NEW; do
    tag=$(basename $lib .so)_$rep
    KGAT_HIP_LIB=$PWD/$lib timeout -k 10 400 python -u bench.py --steps 30 --no-cpu-baseline --no-parity --no-kg-leg \
      > gpurun_out/ab/$tag.log 2>&1 || { tail -20 gpurun_out/ab/$tag.log; exit 1; }
    python3 -c "
import json; r=json.loads(open('gpurun_out/ab/$tag.log').read().strip().splitlines()[-1])
print('$tag', 'full %.4f' % r['ms_per_step'], 'frontier %.4f' % r['frontier_forward']['ms_per_step'], 'tu %.4f' % r['spmm']['table_update']['avg_launch_ms'], 'fwd %.4f' % r['spmm']['fwd_avg_ms'], 'host %.3f' % r['host_launch_ms_per_step'])"
  done
done
