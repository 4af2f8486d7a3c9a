#!/usr/bin/env python3
"""Clock the kept SHA-1 kernel actually runs at (diagnostic build).

    make ablib_sha1 VAR=sha1_clock DEFS="-DCIO_SHA1_CLOCK_DIAG"
    python tools/sha1_clock.py chunkio_amd/lib/ab/sha1_clock.so [--copies 1,8]

The build records, per workgroup, the round wave's s_memtime (shader clock) and
s_memrealtime (100 MHz) at the start and end of its block loop.  For the cfg5
batch (1024 x 409600 B) repeated `copies` times (1 = 32 workgroups on 32 CUs;
8 = 256 workgroups, one per CU), this prints the clock the round waves ran at,
their cycles per round (6401 blocks x 80 rounds), and the issue floor at that
clock beside the 2.40 GHz one bench.py quotes.
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
    ap.add_argument("lib")
    ap.add_argument("--copies", default="1,8")
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    import torch
    import hashlib
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl
    lib = ctypes.CDLL(os.path.abspath(args.lib), mode=ctypes.RTLD_LOCAL)
    lib.cio_sha1_batch_dev.argtypes = [ctypes.c_void_p, U64P, U64P, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    lib.cio_sha1_diag_clock.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lens0 = wl.cfg2_lens()
    offs0 = wl.packed_offsets(lens0)
    dev = torch.empty(wl.batch_bytes(offs0, lens0), dtype=torch.uint8, device="cuda")
    cio.fill_synthetic(dev, offs0, lens0, wl.CFG2_SEED)
    torch.cuda.synchronize()
    blocks = (int(lens0[0]) + 8) // 64 + 1          # 6401 for 409600 B
    for copies in [int(x) for x in args.copies.split(",")]:
        o = np.ascontiguousarray(np.tile(offs0, copies).astype(np.uint64))   # the same bytes, hashed `copies` times
        ln = np.ascontiguousarray(np.tile(lens0, copies).astype(np.uint64))
        n = len(ln)
        out = torch.empty(n * 20, dtype=torch.uint8, device="cuda")
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        per = 8 if n <= 8 * cus else 16 if n <= 16 * cus else 32     # sha1_chunks_per_wg's geometry
        nwg = (n + per - 1) // per
        rows = []
        for it in range(args.iters):
            t0 = time.perf_counter()
            assert lib.cio_sha1_batch_dev(dev.data_ptr(), o.ctypes.data_as(U64P), ln.ctypes.data_as(U64P),
                                          out.data_ptr(), n, None) == 0
            wall = time.perf_counter() - t0
            clk = np.zeros((nwg, 4), dtype=np.uint64)
            assert lib.cio_sha1_diag_clock(clk.ctypes.data, nwg) == 0
            dc = (clk[:, 1] - clk[:, 0]).astype(np.float64)
            dr = (clk[:, 3] - clk[:, 2]).astype(np.float64) * 10.0          # ns
            ghz = dc / dr
            rows.append((wall * 1e3, float(np.median(dr)) / 1e6, float(np.median(ghz)), float(ghz.min()),
                         float(ghz.max()), float(np.median(dc)) / (blocks * 80)))
        d = out[:20].cpu().numpy().tobytes()
        ref = hashlib.sha1(dev[int(offs0[0]):int(offs0[0]) + int(lens0[0])].cpu().numpy().tobytes()).digest()
        for r in rows:
            print("copies %d (%d workgroups): call %.2f ms, round-wave loop %.3f ms, clock %.3f GHz (min %.3f max %.3f), "
                  "%.2f cycles/round; issue floor at this clock %.3f ms (at 2.40 GHz %.3f ms), digest ok %s"
                  % (copies, nwg, r[0], r[1], r[2], r[3], r[4], r[5], blocks * 80 * 20.35 / r[2] / 1e6,
                     blocks * 80 * 20.35 / 2.40 / 1e6, d == ref), flush=True)


if __name__ == "__main__":
    main()
