#!/usr/bin/env python3
"""Pair a bench.py line with the rocprofv3 kernel trace of the SAME run, so
that roofline.frac can be recomputed from the committed profile (VERDICT r2
"Next round" item 1).

    python tools/prof_pair.py <bench.json> <run_kernel_trace.csv> <kernel-substring> [iso]

The timed window is located from the end of the kernel's dispatch list:
bench.py launches the kernel during an untimed device ramp, then `warmup`
times, then `steps` timed launches back to back, then `iso` isolated
diagnostic launches (min(steps, 100) for the CRC lines, 0 for SHA-1).
Prints JSON: the timed window's mean / median kernel duration from rocprof,
the bench line's own event mean, algorithmic bytes / rocprof mean as GB/s and
as a fraction of 8 TB/s, its ratio to the line's roofline.frac, and whether
the rocprof mean fits inside the line's ms_per_step.
"""
import csv
import json
import sys

import numpy as np

PEAK = 8000.0


def main():
    bench_path, trace, name = sys.argv[1], sys.argv[2], sys.argv[3]
    with open(bench_path) as f:
        line = json.loads([x for x in f.read().splitlines() if x.startswith("{")][-1])
    steps, warm = int(line["steps"]), int(line["warmup"])
    iso = int(sys.argv[4]) if len(sys.argv) > 4 else min(steps, 100)
    rows = [r for r in csv.DictReader(open(trace)) if name in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows])
    s = np.array([int(r["Start_Timestamp"]) / 1e3 for r in rows])
    end = len(d)
    a, b = end - iso - steps, end - iso
    x = d[a:b]
    roof = line.get("roofline", {})
    algo = roof.get("algorithmic_bytes_per_launch")
    if algo is None:                       # SHA-1 line: the batch bytes per launch
        algo = int(line["value"] * 1e9 * line["ms_per_step"] * 1e-3 / max(1, line.get("n_gpus", 1)))
    out = {"kernel": name, "dispatches": int(end), "timed_window": [int(a), int(b)],
           "rocprof_mean_us": round(float(x.mean()), 3), "rocprof_median_us": round(float(np.median(x)), 3),
           "rocprof_min_us": round(float(x.min()), 3),
           "start_to_start_us": round(float((s[b - 1] - s[a]) / max(1, b - 1 - a)), 3),
           "bench_kernel_ms_mean": roof.get("kernel_ms_mean"), "bench_ms_per_step": line["ms_per_step"],
           "algorithmic_bytes_per_launch": int(algo)}
    ach = algo / (x.mean() * 1e-6) / 1e9
    out["rocprof_achieved_GBps"] = round(ach, 1)
    out["rocprof_frac_of_8TBps"] = round(ach / PEAK, 4)
    if "frac" in roof:
        out["bench_frac"] = roof["frac"]
        out["rocprof_over_bench_frac"] = round(ach / PEAK / roof["frac"], 4)
    rs = roof.get("read_stream", {}).get("GBps")
    if rs:
        out["same_box_read_stream_GBps"] = rs
        out["rocprof_frac_of_read_stream"] = round(ach / rs, 4)
    out["rocprof_mean_within_ms_per_step"] = bool(x.mean() * 1e-3 <= line["ms_per_step"])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
