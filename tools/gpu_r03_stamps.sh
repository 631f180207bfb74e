#!/bin/bash
# biinter_fwd phase stamps (tools/biinter_stamps): with and without the per-column-block sched_barrier.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/biinter_stamps > gpurun_out/biinter_stamps.log 2>&1 || { tail -5 gpurun_out/biinter_stamps.log; exit 1; }
cat gpurun_out/biinter_stamps.log
