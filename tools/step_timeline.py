"""Print one step's kernel timeline from a rocprofv3 kernel trace: the launches between the n-th and
(n+1)-th occurrence of a marker kernel (default: the layer-0 forward SpMM of width d).
usage: python tools/step_timeline.py <run_kernel_trace.csv> <marker substring> <occurrence index> [<every>]"""
import csv
import sys


def main() -> None:
    path, marker, idx = sys.argv[1], sys.argv[2], int(sys.argv[3])
    every = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    seq = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    marks = [i for i, (n, _, _) in enumerate(seq) if marker in n][::every]
    print(f"{len(marks)} markers")
    a, b = marks[idx], marks[idx + 1] if idx + 1 < len(marks) else len(seq)
    t0 = seq[a][1]
    busy = 0
    for n, s, e in seq[a:b]:
        busy += e - s
        print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:9.1f}  {n[:110]}")
    print(f"span {(seq[b - 1][2] - t0) / 1e3:.1f} us, kernel busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
