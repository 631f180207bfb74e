#!/bin/bash
# bi-interaction forward with W in registers (KGAT_FWD_VARIANT=40) vs the default (8): time + digests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 8 40 8 40; do
  KGAT_FWD_VARIANT=$v timeout -k 10 300 python3 tools/ab_fwd.py gpurun_out/abfwd_$v.json > gpurun_out/abfwd_$v.log 2>&1 || { tail -5 gpurun_out/abfwd_$v.log; exit 1; }
done
python3 tools/ab_fwd.py --compare gpurun_out/abfwd_8.json gpurun_out/abfwd_40.json
