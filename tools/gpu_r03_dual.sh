#!/bin/bash
# Wide bi-interaction GEMM A/B: dual vs separate launches (KGAT_DUAL_GEMM) x stage depth
# (KGAT_GEMM_BK 16 / 32), per-kernel stats of each at 300k and 1M rows (256 -> 256), plus C4's
# 128 -> 128 shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/dual
rm -rf $OUT; mkdir -p $OUT
for shape in "300000 256 256" "1000000 256 256" "1000000 128 128"; do
  set -- $shape
  for v in 0 1; do
    for bk in 16 32; do
      tag=r$1_${2}x${3}_d${v}_k$bk
      KGAT_DUAL_GEMM=$v KGAT_GEMM_BK=$bk timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$tag -o run \
        --output-format csv -- python3 tools/bench_dual.py --rows $1 --din $2 --dout $3 > $OUT/$tag.log 2>&1 \
        || { tail -20 $OUT/$tag.log; exit 1; }
      grep '^{' $OUT/$tag.log
    done
  done
done
echo done
