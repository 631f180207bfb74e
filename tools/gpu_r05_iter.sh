#!/bin/bash
# Round 5 iteration on one GPU: the GPU suite, a short C2 bench line (no CPU baseline / parity / KG legs),
# and a rocprof kernel trace of the same run with one full and one frontier step's timelines.
# usage: tools/gpu_r05_iter.sh TAG [tests] [bench] [prof]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
shift
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
        > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_tests.log | head -30; tail -3 gpurun_out/${TAG}_tests.log; exit 1; }
      tail -1 gpurun_out/${TAG}_tests.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
      tail -2 gpurun_out/${TAG}_smoke.log ;;
    bench)
      timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity --no-kg-leg \
        > gpurun_out/${TAG}_c2_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_c2_bench.log; exit 1; }
      python3 - gpurun_out/${TAG}_c2_bench.log <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
fr = d.get("frontier_forward", {})
print("full ms", round(d["ms_per_step"], 4), "frontier ms", round(fr.get("ms_per_step", 0), 4),
      "bit_identical", fr.get("bit_identical_to_full", {}).get("pass"), "roofline", round(d["roofline"]["frac"], 3))
EOF
      ;;
    benchkg)
      timeout -k 10 900 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity \
        > gpurun_out/${TAG}_c2_benchkg.log 2>&1 || { tail -30 gpurun_out/${TAG}_c2_benchkg.log; exit 1; }
      python3 - gpurun_out/${TAG}_c2_benchkg.log <<'EOF2'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
kg = d.get("kg_refresh", {})
r = kg.get("refresh", {})
print("full ms", round(d["ms_per_step"], 4), "frontier ms", round(d.get("frontier_forward", {}).get("ms_per_step", 0), 4))
print("refresh ms", r.get("ms_per_call"), "edge_scores ms", r.get("edge_scores_avg_ms"), "frac", r.get("roofline", {}).get("frac"),
      "softmax ms", r.get("row_softmax_avg_ms"), "GB/s", r.get("row_softmax_GBps"))
print("kg captured ms", kg.get("captured", {}).get("ms_per_step"), "epoch s", kg.get("epoch_estimate", {}).get("seconds"))
EOF2
      ;;
    prof)
      rm -rf gpurun_out/${TAG}_prof
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
        python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-kg-leg \
        > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
      T=$(find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" | head -1)
      python3 tools/step_timeline.py "$T" bpr_fwd_kernel 5 > gpurun_out/${TAG}_full_step.txt
      python3 tools/step_timeline.py "$T" bpr_fwd_kernel -6 > gpurun_out/${TAG}_frontier_step.txt
      tail -1 gpurun_out/${TAG}_full_step.txt
      tail -1 gpurun_out/${TAG}_frontier_step.txt ;;
    profkg)
      rm -rf gpurun_out/${TAG}_profkg
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_profkg -o run --output-format csv -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-frontier-leg \
        > gpurun_out/${TAG}_profkg.log 2>&1 || { tail -20 gpurun_out/${TAG}_profkg.log; exit 1; }
      S=$(find gpurun_out/${TAG}_profkg -name "*kernel_stats.csv" | head -1)
      cp "$S" gpurun_out/${TAG}_profkg_stats.csv
      grep -E "softmax|score|slot_sum" "$S" | cut -c1-200 ;;
    nfm)
      timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "nfm or NFM" \
        > gpurun_out/${TAG}_nfm_tests.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_nfm_tests.log | head -30; exit 1; }
      tail -1 gpurun_out/${TAG}_nfm_tests.log ;;
    c3prof)
      rm -rf gpurun_out/${TAG}_c3prof
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c3prof -o run --output-format csv -- \
        python3 bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-kg-leg \
        > gpurun_out/${TAG}_c3prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_c3prof.log; exit 1; }
      S=$(find gpurun_out/${TAG}_c3prof -name "*kernel_stats.csv" | head -1)
      grep -E "nfm" "$S" | cut -c1-160
      python3 - gpurun_out/${TAG}_c3prof.log <<'EOF3'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
nf = d.get("nfm", {})
print("c3 ms", round(d["ms_per_step"], 3), "nfm keys", list(nf.keys())[:12])
for k in ("predict", "train"):
    if k in nf:
        print(k, {kk: nf[k][kk] for kk in list(nf[k])[:10]})
EOF3
      ;;
    c5small)
      timeout -k 10 400 python -u bench.py --config c5 --scale 0.02 --rank-share 8 --steps 3 --warmup 1 --no-cpu-baseline \
        > gpurun_out/${TAG}_c5small.log 2>&1 || { tail -30 gpurun_out/${TAG}_c5small.log; exit 1; }
      tail -1 gpurun_out/${TAG}_c5small.log | cut -c1-400 ;;
    hostprof)
      timeout -k 10 300 python3 tools/host_profile.py > gpurun_out/${TAG}_host.txt 2>&1 || { tail -20 gpurun_out/${TAG}_host.txt; exit 1; }
      timeout -k 10 300 python3 tools/host_profile.py --full > gpurun_out/${TAG}_host_full.txt 2>&1 || { tail -20 gpurun_out/${TAG}_host_full.txt; exit 1; }
      grep "ms/step" gpurun_out/${TAG}_host.txt gpurun_out/${TAG}_host_full.txt ;;
  esac
done
echo done
