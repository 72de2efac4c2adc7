#!/usr/bin/env python3
"""Convert framework profiles into one Chrome trace (reference tools/timeline.py).

    python tools/timeline.py --profile_path trainer0=/tmp/p0,trainer1=/tmp/p1 --timeline_path /tmp/timeline

A profile is the JSON written by ``fluid.profiler.stop_profiler(profile_path=...)``
(host op ranges per thread and, with the GPU state, the device ranges of every op
on the HIP device clock).  Open the result in chrome://tracing or Perfetto.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    from paddle_amd.utils.profiler import chrome_trace

    ap = argparse.ArgumentParser()
    ap.add_argument("--profile_path", default="/tmp/profile")
    ap.add_argument("--timeline_path", default="/tmp/timeline")
    a = ap.parse_args(argv)
    profiles = {}
    paths = a.profile_path.split(",")
    for item in paths:
        k, path = item.split("=", 1) if "=" in item else ("trainer", item)
        with open(path) as f:
            profiles[k] = json.load(f)
    with open(a.timeline_path, "w") as f:
        f.write(chrome_trace(profiles))
    return a.timeline_path


if __name__ == "__main__":
    main()
