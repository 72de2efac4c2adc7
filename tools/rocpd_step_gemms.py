#!/usr/bin/env python3
"""List the kernels of the LAST training step in a rocprofv3 kernel-trace DB in
launch order (step boundary = the last dispatch whose name contains MARKER), with
the grid (workgroups) and duration: per-shape attribution of the GEMM/conv time.

    python tools/rocpd_step_gemms.py run_results.db MARKER [filter-regex] [markers-per-step]
"""
import re
import sqlite3
import sys


def main():
    db, marker = sys.argv[1], sys.argv[2]
    filt = re.compile(sys.argv[3]) if len(sys.argv) > 3 else None
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start"))
    idx = [i for i, r in enumerate(rows) if marker in r[0]]
    k = int(sys.argv[4]) if len(sys.argv) > 4 else 1  # markers per step
    step = rows[idx[-k]:]
    tot = sum(r[2] - r[1] for r in step)
    print(f"last step: {len(step)} kernels, kernel time {tot / 1e6:.2f} ms, wall {(step[-1][2] - step[0][1]) / 1e6:.2f} ms")
    for r in step:
        if filt is None or filt.search(r[0]):
            m = re.search(r"(\w+)<([^>]*)>", r[0])
            nm = (m.group(1) + "<" + m.group(2).replace(" ", "") + ">") if m else r[0][:50]
            print(f"{nm[:70]:70s} wg={r[3] // max(r[4], 1):6d} {(r[2] - r[1]) / 1e3:8.1f} us")


if __name__ == "__main__":
    main()
