#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--kernel-trace`` SQLite output (``*_results.db``) into a
markdown table: per-kernel total / calls / average, optionally per step.

    python tools/rocpd_summary.py gpurun_out/prof3/run_results.db "title" [steps] [top]
"""
import sqlite3
import sys
from collections import defaultdict


def summarize(db, title, steps=None, top=40):
    c = sqlite3.connect(db)
    agg = defaultdict(lambda: [0, 0.0])
    for name, dur in c.execute("select name, duration from kernels"):
        a = agg[name]
        a[0] += 1
        a[1] += dur
    tot = sum(v[1] for v in agg.values())
    per = f" over {steps} steps ({tot / 1e6 / steps:.1f} ms/step)" if steps else ""
    out = [f"# {title}", "", f"source: `{db}` (rocprofv3 --kernel-trace)", "",
           f"total GPU kernel time: {tot / 1e6:.1f} ms{per}", "",
           "| rank | total ms | % | calls | avg us | kernel |", "|---|---|---|---|---|---|"]
    for i, (n, (k, d)) in enumerate(sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]):
        out.append(f"| {i + 1} | {d / 1e6:.1f} | {100 * d / tot:.1f} | {k} | {d / k / 1e3:.1f} | `{n[:110]}` |")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    print(summarize(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else None,
                    int(sys.argv[4]) if len(sys.argv) > 4 else 40))
