"""Write a rocprofv3 --stats kernel summary (markdown) for profiles/.

usage: python tools/prof_summary.py <run_kernel_stats.csv> <out.md> "<command line>" [steps]
"""
import csv
import sys


def main() -> None:
    src, out, cmd = sys.argv[1], sys.argv[2], sys.argv[3]
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 12
    cfg = sys.argv[5] if len(sys.argv) > 5 else "C2"
    rows = list(csv.DictReader(open(src)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"# rocprofv3 --kernel-trace --stats -- {cmd} ({cfg}, 1x MI355X)",
             f"# {steps} CF steps profiled (warm-up + timed); avg per launch; per-step = total / {steps}", "",
             "| kernel | calls | avg us | us / step | % |", "|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        t = float(r["TotalDurationNs"])
        if t / tot < 0.001:
            continue
        lines.append(f"| `{r['Name'][:96]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{t / 1e3 / steps:.1f} | {100 * t / tot:.1f} |")
    lines.append(f"\nkernel time per step: {tot / 1e3 / steps:.0f} us")
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
