"""Average per-dispatch counter values per (run directory, kernel) under a rocprofv3 output tree.

    python tools/pmc_dump.py <dir> [kernel-substring]
"""
import csv
import glob
import sys
from collections import defaultdict
from pathlib import Path


def main():
    src = Path(sys.argv[1])
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(str(src / "**" / "*counter_collection.csv"), recursive=True)):
        run = Path(f).relative_to(src).parts[0]
        for row in csv.DictReader(open(f)):
            if sub in row["Kernel_Name"]:
                vals[(run, row["Kernel_Name"][:60])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for (run, k), c in sorted(vals.items()):
        print(f"[{run}] {k}")
        for name, v in sorted(c.items()):
            print(f"   {name:28s} {sum(v) / len(v):16.1f}")


if __name__ == "__main__":
    main()
