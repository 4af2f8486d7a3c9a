#!/usr/bin/env python3
"""Kernel durations from a rocprofv3 --kernel-trace CSV, per phase of bench.py.

    python tools/prof_window.py <run_kernel_trace.csv> <warmup> <steps> [kernel-substring]

bench.py launches the CRC kernel during an untimed device ramp, then `warmup`
times, then `steps` timed launches back to back, then min(steps, 100)
isolated diagnostic launches (phases are located from the end).  Prints the
mean / median / min duration of each phase (dispatches in start order) so the
timed window can be compared with bench.py's `kernel_ms_mean`.
"""
import csv
import json
import sys

import numpy as np


def main():
    path, warm, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    name = sys.argv[4] if len(sys.argv) > 4 else "crc32_stream_kernel"
    rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows])
    s = np.array([int(r["Start_Timestamp"]) / 1e3 for r in rows])
    out = {"kernel": name, "dispatches": len(d)}
    # Counted from the end: bench.py's untimed device ramp (a variable number
    # of launches) precedes the warmup steps.
    iso = min(steps, 100)
    end = len(d)
    phases = {"ramp": (0, max(0, end - iso - steps - warm)),
              "warmup": (max(0, end - iso - steps - warm), end - iso - steps),
              "timed": (end - iso - steps, end - iso), "isolated": (end - iso, end)}
    for k, (a, b) in phases.items():
        x = d[a:b]
        if len(x):
            out[k] = {"n": int(len(x)), "mean_us": round(float(x.mean()), 2),
                      "median_us": round(float(np.median(x)), 2), "min_us": round(float(x.min()), 2)}
    a, b = phases["timed"]
    if b - a > 1 and b <= len(s):
        out["timed"]["start_to_start_us"] = round(float((s[b - 1] - s[a]) / (b - 1 - a)), 2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
