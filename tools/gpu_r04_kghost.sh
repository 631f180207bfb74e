#!/bin/bash
# Host profile + kernel trace of the captured KG step (KGAT.capture_kg_step) vs the eager lazy step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_profile.py --kg --captured > gpurun_out/r04_kg_captured_host.log 2>&1 || { tail -30 gpurun_out/r04_kg_captured_host.log; exit 1; }
head -45 gpurun_out/r04_kg_captured_host.log | grep -v "^$" | head -40
timeout -k 10 300 python -u tools/host_profile.py --kg --lazy > gpurun_out/r04_kg_lazy_host.log 2>&1 || { tail -30 gpurun_out/r04_kg_lazy_host.log; exit 1; }
head -3 gpurun_out/r04_kg_lazy_host.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_prof_kg -o run --output-format csv -- \
  python3 tools/host_profile.py --kg --captured > gpurun_out/r04_prof_kg.log 2>&1 || { tail -20 gpurun_out/r04_prof_kg.log; exit 1; }
echo done
