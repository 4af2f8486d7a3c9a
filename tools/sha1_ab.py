#!/usr/bin/env python3
"""In-process A/B of cio_sha1_batch_dev across builds of libchunkio_amd.so.

    python tools/sha1_ab.py --libs chunkio_amd/lib/libchunkio_amd.so,chunkio_amd/lib/ab/x.so [--rounds 5]

One cfg2-shaped batch (1024 x 409600 B, generated in HBM) is hashed by every
library in turn, rounds interleaved so clock drift hits all of them; digests
must be identical across libraries.  Each call is timed on the host around a
synchronous cio_sha1_batch_dev (the call synchronises its stream).
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

U64P = ctypes.POINTER(ctypes.c_uint64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--chunks", type=int, default=0, help="hash only the first N chunks of the batch")
    ap.add_argument("--diag", action="store_true",
                    help="timing only: diagnostic builds (CIO_SHA1_DIAG_*) give wrong digests on purpose")
    args = ap.parse_args()
    import torch
    import hashlib
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl
    libs = []
    for p in args.libs.split(","):
        lib = ctypes.CDLL(os.path.abspath(p), mode=ctypes.RTLD_LOCAL)
        lib.cio_sha1_batch_dev.argtypes = [ctypes.c_void_p, U64P, U64P, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_void_p]
        libs.append((p, lib))
    lens = wl.cfg2_lens()
    offs = wl.packed_offsets(lens)
    if args.chunks:
        lens, offs = lens[:args.chunks], offs[:args.chunks]
    dev = torch.empty(wl.batch_bytes(offs, lens), dtype=torch.uint8, device="cuda")
    cio.fill_synthetic(dev, offs, lens, wl.CFG2_SEED)
    o = np.ascontiguousarray(offs.astype(np.uint64))
    ln = np.ascontiguousarray(lens.astype(np.uint64))
    out = torch.empty(len(lens) * 20, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()

    def call(lib):
        rc = lib.cio_sha1_batch_dev(dev.data_ptr(), o.ctypes.data_as(U64P), ln.ctypes.data_as(U64P),
                                    out.data_ptr(), len(lens), None)
        assert rc == 0

    digests = []
    for _, lib in libs:
        call(lib)
        digests.append(out.cpu().numpy().copy())
    for d in digests[1:] if not args.diag else []:
        assert np.array_equal(d, digests[0]), "digests differ between libraries"
    for i in sorted({0, 1, len(lens) // 2, len(lens) - 1}):   # hashlib (OpenSSL) spot check of the common result
        want = hashlib.sha1(wl.gen_chunk(wl.CFG2_SEED, i, int(lens[i])).tobytes()).digest()
        assert digests[0][20 * i:20 * i + 20].tobytes() == want, i
    times = {p: [] for p, _ in libs}
    for _ in range(args.rounds):
        for p, lib in libs:
            call(lib)
            t0 = time.perf_counter()
            for _ in range(args.iters):
                call(lib)
            times[p].append((time.perf_counter() - t0) / args.iters * 1e3)
    total = int(lens.sum())
    for p, _ in libs:
        t = np.array(times[p])
        print(f"{os.path.basename(p):28s} ms/call median {np.median(t):.3f} min {t.min():.3f} "
              f"-> {total / np.median(t) / 1e6:.2f} GB/s  rounds {np.round(t, 3).tolist()}")
    print("digests equal across libraries:", "not checked (--diag)" if args.diag else True,
          "; hashlib spot checks of the first library: True")


if __name__ == "__main__":
    main()
