"""Per-stream busy time of one traced C4 step with the pipelined owner exchange (bench.py --config c4
--exchange-at-1 --dp sharded under rocprofv3 --kernel-trace): the step window runs from one bpr_fwd_kernel
launch to the next; for every stream the summed kernel time inside the window, and the tail -- the time
from the last main-stream backward kernel to the window's last kernel end (the exposed owner chain).

usage: python3 tools/c4_exchange_trace.py run_kernel_trace.csv [step index, default: the last full one]
"""
import collections
import csv
import sys


def main() -> int:
    rows = list(csv.DictReader(open(sys.argv[1])))
    for r in rows:
        r["t0"], r["t1"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["t0"])
    marks = [r["t0"] for r in rows if "bpr_fwd_kernel" in r["Kernel_Name"]]
    if len(marks) < 2:
        print("fewer than two bpr_fwd_kernel launches")
        return 1
    k = int(sys.argv[2]) if len(sys.argv) > 2 else len(marks) - 2
    lo, hi = marks[k], marks[k + 1]
    win = [r for r in rows if lo <= r["t0"] < hi]
    busy = collections.defaultdict(int)
    names = collections.defaultdict(collections.Counter)
    for r in win:
        busy[r["Stream_Id"]] += r["t1"] - r["t0"]
        names[r["Stream_Id"]][r["Kernel_Name"].split("(")[0][:60]] += r["t1"] - r["t0"]
    main_stream = max(busy, key=lambda s: busy[s])
    end = max(r["t1"] for r in win)
    print(f"step {k}: window {(hi - lo) / 1e6:.3f} ms (bpr_fwd to bpr_fwd), last kernel end "
          f"{(end - lo) / 1e6:.3f} ms")
    for s, b in sorted(busy.items(), key=lambda x: -x[1]):
        top = ", ".join(f"{n} {t / 1e6:.2f}" for n, t in names[s].most_common(4))
        print(f"  stream {s}{' (main)' if s == main_stream else ''}: {b / 1e6:.3f} ms busy, "
              f"{sum(1 for r in win if r['Stream_Id'] == s)} kernels; top: {top}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
