#!/bin/bash
# C5 rehearsal at 2 ranks on this one GPU (gloo, host-staged transport): one step's pipelined-forward
# block marks per rank (bench.py --timeline -> gpurun_out/c5_timeline_rank*.txt).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp KGAT_BENCH_BACKEND=gloo
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --config c5 --scale 0.01 --steps 3 --warmup 1 --no-frontier-leg \
  --no-cpu-baseline --no-parity --timeline > gpurun_out/r04_c5_timeline.log 2>&1 || { tail -30 gpurun_out/r04_c5_timeline.log; exit 1; }
tail -1 gpurun_out/r04_c5_timeline.log | cut -c1-300
cat gpurun_out/c5_timeline_rank0.txt
