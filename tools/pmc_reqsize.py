#!/usr/bin/env python3
"""HBM read bytes per launch from the L2's memory-side request counters split
by size, with no calibration factor:

    rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum \
        TCC_EA0_RDREQ_128B_sum -d DIR -o run --output-format csv -- python3 bench.py ...
    python tools/pmc_reqsize.py DIR [--algo BYTES]

read bytes = 32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B (4 TCC slots,
one pass).  The request total checks that the three sizes partition every
request.  FETCH_SIZE (rocprofv3's derived counter) tallies a 128-byte request
at 64 bytes on gfx950 (MI355X_MICROARCH.md, HBM), which tools/pmc_traffic.py
corrects with a x2 that is exact only when every request is 128 bytes; this
pass needs no such assumption.
"""
import csv
import glob
import json
import os
import sys

KERNELS = ("crc32_stream_kernel", "crc32_small_kernel", "sha1_kernel")
COUNTERS = ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")


def main():
    d = sys.argv[1]
    algo = int(sys.argv[sys.argv.index("--algo") + 1]) if "--algo" in sys.argv else None
    per = {}
    kern = set()
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                k = next((k for k in KERNELS if k in name), None)
                if k is None or row.get("Counter_Name") not in COUNTERS:
                    continue
                kern.add(k)
                key = row.get("Dispatch_Id") or row.get("Correlation_Id")
                per.setdefault(key, {}).setdefault(row["Counter_Name"], 0.0)
                per[key][row["Counter_Name"]] += float(row["Counter_Value"])
    if not per:
        sys.exit("no request-size rows for " + "/".join(KERNELS))
    n = len(per)
    mean = {c: sum(v.get(c, 0.0) for v in per.values()) / n for c in COUNTERS}
    tot, r32, r64, r128 = (mean[c] for c in COUNTERS)
    read_b = 32 * r32 + 64 * r64 + 128 * r128
    out = {"kernel": "/".join(sorted(kern)), "dispatches": n,
           "rdreq": round(tot), "rdreq_32b": round(r32), "rdreq_64b": round(r64), "rdreq_128b": round(r128),
           "sizes_cover_all_requests": abs((r32 + r64 + r128) - tot) <= 1e-6 * max(tot, 1.0),
           "read_bytes_per_launch": int(read_b),
           "method": "32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B per launch (no calibration factor)"}
    if algo:
        out["algorithmic_bytes_per_launch"] = algo
        out["read_over_algorithmic"] = round(read_b / algo, 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
