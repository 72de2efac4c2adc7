"""Summarise rocprofv3 counter-collection CSVs: per kernel name, the mean of each
counter over dispatches (plus duration from the kernel trace when present).
usage: pmc_summary.py <rocprofv3 output dir> [kernel-substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            if sub and sub not in k:
                continue
            vals[k[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in vals.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"  {c:32s} mean={sum(v)/len(v):.4g} n={len(v)}")


if __name__ == "__main__":
    main()
