#!/usr/bin/env python3
"""Config-1 loop (1000 files x 5 x 400 KB) through the C chunk layer with the
CRC off, per write (immediate), deferred with GPU batched syncs, and deferred
on the host pool: how much of the loop the CRC costs at all.

    python tools/perf_ceiling.py [--rounds R] [--batch B]
"""
import argparse
import os
import shutil
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--legs", default="nocrc,immediate,deferred,deferred_async,deferred_host,deferred_async_host")
    args = ap.parse_args()
    import chunkio_amd as cio
    from chunkio_amd import chunkfile as cf
    d400 = open(os.path.join(ROOT, "tests", "golden", "400kb.txt"), "rb").read()
    legs = {"nocrc": (0, None), "immediate": (cf.CIO_CHECKSUM, None),
            "deferred": (cf.CIO_CHECKSUM | cf.CIOA_DEFERRED_CRC, None),
            "deferred_async": (cf.CIO_CHECKSUM | cf.CIOA_DEFERRED_CRC | cf.CIOA_BENCH_PIPELINED_SYNC, None),
            "deferred_host": (cf.CIO_CHECKSUM | cf.CIOA_DEFERRED_CRC, 16),
            "deferred_async_host": (cf.CIO_CHECKSUM | cf.CIOA_DEFERRED_CRC | cf.CIOA_BENCH_PIPELINED_SYNC, 16)}
    res = {k: [] for k in args.legs.split(",")}
    root = tempfile.mkdtemp(prefix="cioa-ceil-")
    try:
        for r in range(args.rounds + 1):
            for k in res:
                flags, threads = legs[k]
                if threads:
                    cio.route(reset=True, threads=threads)
                path = os.path.join(root, k)
                secs, nb = cf.perf_write(path, d400, 1000, 5, args.batch, flags)
                cio.route(reset=True)
                with open(os.path.join(path, "test-perf", "perf-test-0999.txt"), "rb") as f:
                    hdr = f.read(10).hex()
                shutil.rmtree(path)
                if r:
                    res[k].append(nb / secs / 1e9)
                print(f"round {r} {k:15s} {nb / secs / 1e9:6.3f} GB/s  header {hdr}", flush=True)
    finally:
        shutil.rmtree(root, ignore_errors=True)
    for k, v in res.items():
        print(f"{k:15s} best {max(v):.3f} median {sorted(v)[len(v) // 2]:.3f} GB/s")


if __name__ == "__main__":
    main()
