#!/bin/bash
# A/B of the bi-interaction forward variants (KGAT_FWD_VARIANT): the first is the baseline.
# usage: tools/gpu_ab_fwd.sh 8 24 40 ...
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_fwd.log
for v in "$@"; do
  KGAT_FWD_VARIANT=$v timeout -k 10 200 python -u tools/ab_fwd.py gpurun_out/fwd_$v.json >> gpurun_out/ab_fwd.log 2>&1 || { tail -20 gpurun_out/ab_fwd.log; exit 1; }
done
for v in "${@:2}"; do
  echo "== $1 vs $v" >> gpurun_out/ab_fwd.log
  python tools/ab_fwd.py --compare gpurun_out/fwd_$1.json gpurun_out/fwd_$v.json >> gpurun_out/ab_fwd.log 2>&1
done
grep -A8 "==" gpurun_out/ab_fwd.log
