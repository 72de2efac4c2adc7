#!/usr/bin/env python3
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output: kernel, VGPRs, AGPRs, scratch, LDS, occupancy."""
import re, subprocess, sys

def main(src, extra=()):
    cmd = ["hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-c", src, "-o", "/dev/null",
           "-Rpass-analysis=kernel-resource-usage", *extra]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    cur = None
    rows = []
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        for key in ("VGPRs", "AGPRs", "ScratchSize \\[bytes/lane\\]", "LDS Size \\[bytes/block\\]", "Occupancy \\[waves/SIMD\\]"):
            m = re.search(key + r": (\d+)", line)
            if m and cur is not None:
                cur[key.split()[0]] = int(m.group(1))
        if "error" in line:
            print(line)
    for r in rows:
        n = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
        print(f"v{r.get('VGPRs')} a{r.get('AGPRs')} scr{r.get('ScratchSize')} lds{r.get('LDS')} occ{r.get('Occupancy')}  {n[:150]}")

if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
