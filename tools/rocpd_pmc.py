#!/usr/bin/env python3
"""Per-kernel PMC counter totals from a rocprofv3 --pmc SQLite output.

    python tools/rocpd_pmc.py gpurun_out/pmc1/run_results.db [kernel-substring]
"""
import sqlite3
import sys
from collections import defaultdict


def main(db, filt=None):
    c = sqlite3.connect(db)
    agg = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    for name, counter, value, disp in c.execute(
            "select kernel_name, counter_name, value, dispatch_id from counters_collection"):
        if filt and filt not in name:
            continue
        agg[name][counter] += value
        n[name].add(disp)
    for k, cs in agg.items():
        print(f"{k[:100]}  (dispatches: {len(n[k])})")
        for cn, v in sorted(cs.items()):
            print(f"    {cn:28s} {v / max(1, len(n[k])):16.4g} per dispatch")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
