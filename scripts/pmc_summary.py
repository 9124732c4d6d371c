"""Per-kernel averages of every counter in a rocprofv3 --pmc output directory (CSV mode).

    python scripts/pmc_summary.py <dir> [kernel-substring]
"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row.get("Kernel_Name", "")
            if want in k:
                acc[(k[:90], row["Counter_Name"])].append(float(row["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        print(f"{k:90s} {c:28s} n={len(v):3d} avg={sum(v) / len(v):.6g}")


if __name__ == "__main__":
    main()
