#!/usr/bin/env python3
"""Turn rocprofv3 --pmc CSVs into HBM bytes per launch of the CRC kernel.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> [cfg] [--algo BYTES]

FETCH_SIZE and WRITE_SIZE are collected in separate passes (they do not fit
one TCC pass on gfx950).  Both are in KiB.  Per MI355X_MICROARCH.md (HBM):
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming
read, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for
16-B-per-lane stores and uncalibrated for the kernel's few 4/8-byte stores.
Writes profiles/pmc_<cfg>.json (read by bench.py for roofline.traffic).
"""
import csv
import glob
import json
import os
import sys

# the main kernel a bench config launches (one per run)
KERNELS = ("crc32_stream_kernel", "crc32_small_kernel", "sha1_kernel")


kern_seen = set()


def per_dispatch(d, counter):
    vals = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                if not any(k in name for k in KERNELS):
                    continue
                kern_seen.add(next(k for k in KERNELS if k in name))
                if row.get("Counter_Name") != counter:
                    continue
                key = row.get("Dispatch_Id") or row.get("Correlation_Id")
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    cfg = sys.argv[3] if len(sys.argv) > 3 else "cfg2"
    algo = int(sys.argv[sys.argv.index("--algo") + 1]) if "--algo" in sys.argv else 419430400
    fetch = per_dispatch(fdir, "FETCH_SIZE")
    write = per_dispatch(wdir, "WRITE_SIZE")
    if not fetch:
        sys.exit("no FETCH_SIZE rows for " + "/".join(KERNELS))
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write) if write else 0.0
    read_b = 2.0 * f_kib * 1024.0          # gfx950 correction: FETCH_SIZE = 1/2 of streamed bytes
    write_b = w_kib * 1024.0
    out = {"kernel": "/".join(sorted(kern_seen)), "dispatches": len(fetch),
           "fetch_size_kib_raw": round(f_kib, 1), "write_size_kib_raw": round(w_kib, 1),
           "read_bytes_per_launch": int(read_b), "write_bytes_per_launch": int(write_b),
           "hbm_bytes_per_launch": int(read_b + write_b), "algorithmic_bytes_per_launch": algo,
           "traffic_over_algorithmic": round((read_b + write_b) / algo, 4),
           "correction": "read = 2 x FETCH_SIZE x 1024 (MI355X_MICROARCH.md HBM, gfx950)"}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "profiles", f"pmc_{cfg}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
