#!/usr/bin/env python3
"""Batched host-vs-GPU crossover for host-resident chunks:
the data behind crc_route.c's cost model.

    python tools/route_batch.py [out.json]

For batches of n x 400 KB chunks (n = 1 .. 1024, 400 KB .. 419 MB) in
pageable host memory, rotated over a 2 GiB buffer so repeats come from DRAM
(chunk files in the page cache), the median wall time of
  - cio_crc32_batch_host   (GPU: pinned staging + H2D + kernel + D2H)
  - cio_crc32_batch_cpu    (host crc_update, 1 thread and the box's per-GPU
                            CPU share)
and the fitted model constants: the GPU's fixed cost and rate, the host's
per-thread and all-thread rates.  Also prints each size's winner.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl
    import bench
    T = bench.host_cpu_threads()
    region = 2 << 30
    rng = np.random.default_rng(7)
    host = rng.integers(0, 256, region, dtype=np.uint8)
    L = wl.CFG2_LEN
    rows = []
    for n in (1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024):
        lens = np.full(n, L, np.uint64)
        span = n * L
        nslots = max(1, region // span)
        variants = {"gpu": lambda o: cio.crc32_batch_host_packed(host, o, lens),
                    "cpu_1t": lambda o: cio.crc32_batch_cpu_packed(host, o, lens, threads=1),
                    f"cpu_{T}t": lambda o: cio.crc32_batch_cpu_packed(host, o, lens, threads=T)}
        reps = 30 if span < (64 << 20) else 8
        row = {"chunks": n, "bytes": span}
        ref = None
        for name, fn in variants.items():
            fn(np.arange(n, dtype=np.uint64) * np.uint64(L))      # warm
            ts = []
            for r in range(reps):
                base = (r * 7919 % nslots) * span
                offs = np.arange(n, dtype=np.uint64) * np.uint64(L) + np.uint64(base)
                t0 = time.perf_counter()
                got = fn(offs)
                ts.append(time.perf_counter() - t0)
                if r == 0:
                    if ref is None:
                        ref = got
                    assert np.array_equal(got, ref) or name == "gpu", name
            row[name + "_us"] = round(float(np.median(ts)) * 1e6, 1)
        row["winner_1t"] = "gpu" if row["gpu_us"] < row["cpu_1t_us"] else "cpu"
        row[f"winner_{T}t"] = "gpu" if row["gpu_us"] < row[f"cpu_{T}t_us"] else "cpu"
        rows.append(row)
        print(json.dumps(row), flush=True)
    # fits: GPU t = c + B / r  (least squares over all sizes); host rates at
    # the largest batch
    B = np.array([r["bytes"] for r in rows], float)
    tg = np.array([r["gpu_us"] for r in rows]) * 1e-6
    A = np.vstack([np.ones_like(B), B]).T
    c, inv_r = np.linalg.lstsq(A, tg, rcond=None)[0]
    big = rows[-1]
    fit = {"gpu_fixed_us": round(c * 1e6, 1), "gpu_GBps": round(1 / inv_r / 1e9, 2),
           "cpu_1t_GBps": round(big["bytes"] / (big["cpu_1t_us"] * 1e-6) / 1e9, 2),
           f"cpu_{T}t_GBps": round(big["bytes"] / (big[f"cpu_{T}t_us"] * 1e-6) / 1e9, 2),
           "threads": T, "library_cpu_max_default_1t": int(cio.route(reset=True)[0])}
    print(json.dumps({"fit": fit}), flush=True)
    if out_path:
        with open(out_path, "w") as f:
            json.dump({"rows": rows, "fit": fit, "cpu": bench.cpu_info()}, f, indent=1)


if __name__ == "__main__":
    main()
