"""Split a rocprofv3 kernel trace into segments at the long idle gaps (e.g. the rank shares of one
`bench.py --rank-share K --share-rank a,b` process: the next share's host-side shard build leaves the GPU idle
for seconds) and print per-segment kernel statistics as markdown.
usage: python tools/trace_segments.py run_kernel_trace.csv [min_gap_s] [top] > stats.md"""
import csv
import sys
from collections import defaultdict


def _name(n: str) -> str:
    """The kernel name without its parameter list (the first '(' outside template brackets)."""
    depth = 0
    for i, ch in enumerate(n):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0 and i > 0 and n[i - 1] not in " :":
            return n[:i]
    return n


def main():
    path = sys.argv[1]
    gap = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    segs, cur, last_end = [], [], None
    for s, e, n in rows:
        if last_end is not None and s - last_end > gap * 1e9:
            segs.append(cur)
            cur = []
        cur.append((s, e, n))
        last_end = max(last_end or 0, e)
    segs.append(cur)
    for i, seg in enumerate(segs):
        st = defaultdict(lambda: [0, 0.0])
        for s, e, n in seg:
            st[n][0] += 1
            st[n][1] += (e - s) / 1e3
        busy = sum(v[1] for v in st.values())
        span = (seg[-1][1] - seg[0][0]) / 1e3
        print(f"## segment {i}: {len(seg)} dispatches, kernel busy {busy / 1e3:.1f} ms over a {span / 1e3:.1f} ms span\n")
        print("| kernel | calls | total ms | avg us | % |")
        print("|---|---|---|---|---|")
        for n, (c, t) in sorted(st.items(), key=lambda kv: -kv[1][1])[:top]:
            short = _name(n)[:110]
            print(f"| `{short}` | {c} | {t / 1e3:.2f} | {t / c:.1f} | {100 * t / busy:.1f} |")
        print()


if __name__ == "__main__":
    main()
