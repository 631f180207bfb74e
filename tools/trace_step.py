"""Print one CF step's kernel timeline (gap before, duration) from a rocprofv3 kernel trace.

usage: python tools/trace_step.py <run_kernel_trace.csv> [anchor kernel substring, default adam_multi]
"""
import csv
import sys


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    anchor = sys.argv[2] if len(sys.argv) > 2 else "adam_multi"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    a, b = idx[-3], idx[-2]
    prev = int(rows[a]["End_Timestamp"])
    busy = gaps = 0.0
    for r in rows[a + 1:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"gap {(s - prev) / 1e3:7.1f}  dur {(e - s) / 1e3:7.1f}  {r['Kernel_Name'][:90]}")
        gaps += max(0, s - prev) / 1e3
        busy += (e - s) / 1e3
        prev = e
    print(f"step {(int(rows[b]['End_Timestamp']) - int(rows[a]['End_Timestamp'])) / 1e3:.1f} us: "
          f"kernels {busy:.1f} us, gaps {gaps:.1f} us")


if __name__ == "__main__":
    main()
