#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel_stats.csv into a markdown table."""
import csv, sys

def main(path, title, steps=None, top=30):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = [f"# {title}", "", f"source: `{path}` (rocprofv3 --kernel-trace --stats)", "",
           f"total GPU kernel time: {tot/1e6:.1f} ms" + (f" over {steps} steps ({tot/1e6/steps:.1f} ms/step)" if steps else ""), "",
           "| rank | total ms | % | calls | avg us | kernel |", "|---|---|---|---|---|---|"]
    for i, r in enumerate(sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]):
        out.append(f"| {i+1} | {float(r['TotalDurationNs'])/1e6:.1f} | {float(r['Percentage']):.1f} | {r['Calls']} | "
                   f"{float(r['AverageNs'])/1e3:.1f} | `{r['Name'][:120]}` |")
    return "\n".join(out) + "\n"

if __name__ == "__main__":
    print(main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else None))
