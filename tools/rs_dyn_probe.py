#!/usr/bin/env python3
"""Does a dynamic tail recover the per-CU finish spread of the read-only
stream?  (Go/no-go for dynamic balancing in the CRC kernel.)

    python tools/rs_dyn_probe.py [rounds] ["static;100,4,64;..."]

Over the cfg2 batch (1024 x 409,600 B, 4 rotating buffers): the static
read-only stream (read_stream_kernel, the CRC kernel's split) against
read_stream_dyn_kernel (CIO_GPU_RS_DYN = pool permille, unit steps,
counters), interleaved, every launch bracketed by its own event pair around
the kernel alone (the counter reset is outside the pair).  Mean / median us.

The dynamic kernel is not in the product library (round 5): build
`make ablib VAR=rsdyn DEFS=-DCIO_DIAG_RS_DYN` and run with
CIO_AMD_LIB=chunkio_amd/lib/ab/rsdyn.so.
"""
import ctypes
import os
os.environ.setdefault("CIO_GPU_DIAG", "1")   # the library honours its A/B switches only with this
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    import torch
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl
    lib = cio.lib()
    f = lib.cioa_debug_read_stream_events
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    lens = wl.cfg2_lens()
    offs = wl.packed_offsets(lens, align=16)
    total = int(wl.batch_bytes(offs, lens))
    bufs = [torch.empty(total + 64, dtype=torch.uint8, device=dev) for _ in range(4)]
    for b, t in enumerate(bufs):
        cio.fill_synthetic(t, offs, lens, 0x11 + b)
    sp = torch.cuda.current_stream().cuda_stream
    variants = (sys.argv[2].split(";") if len(sys.argv) > 2 else
                ["", "100,4,64", "150,4,64", "200,4,64", "150,2,64", "150,8,64", "150,4,256", "300,4,64"])
    variants = ["" if v == "static" else v for v in variants]
    res = {v: [] for v in variants}
    n = 100
    for r in range(rounds):
        for v in variants:
            if v:
                os.environ["CIO_GPU_RS_DYN"] = v
            else:
                os.environ.pop("CIO_GPU_RS_DYN", None)
            for i in range(8):
                lib.cio_gpu_read_stream(bufs[i % 4].data_ptr(), total, sp)
            evs = [(lib.cio_gpu_event_create(), lib.cio_gpu_event_create()) for _ in range(n)]
            for i in range(n):
                assert f(bufs[i % 4].data_ptr(), total, sp, evs[i][0], evs[i][1]) == 0
            torch.cuda.synchronize()
            us = np.array([lib.cio_gpu_event_elapsed_ms(a, b) for a, b in evs]) * 1e3
            for a, b in evs:
                lib.cio_gpu_event_destroy(a)
                lib.cio_gpu_event_destroy(b)
            res[v].append(us)
            print(f"round {r} {v or 'static':>10}: mean {us.mean():7.2f} us  median {np.median(us):7.2f}  "
                  f"{(total // 4096 * 4096) / us.mean() / 1e3:7.1f} GB/s", flush=True)
    os.environ.pop("CIO_GPU_RS_DYN", None)
    print("summary (median of round means):")
    for v in variants:
        m = float(np.median([x.mean() for x in res[v]]))
        print(f"  {v or 'static':>10}: {m:7.2f} us  {(total // 4096 * 4096) / m / 1e3:7.1f} GB/s")


if __name__ == "__main__":
    main()
