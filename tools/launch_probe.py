#!/usr/bin/env python3
"""Host launch cost and back-to-back throughput of the CRC kernel (cfg2)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl
    dev = torch.device("cuda:0")
    lib = cio.lib()
    lens = wl.cfg2_lens()
    offs = wl.packed_offsets(lens, align=16)
    total = wl.batch_bytes(offs, lens)
    bufs = [torch.empty(total + 64, dtype=torch.uint8, device=dev) for _ in range(4)]
    for b, t in enumerate(bufs):
        cio.fill_synthetic(t, offs, lens, 7 + b)
    outs = [torch.empty(1024, dtype=torch.int32, device=dev) for _ in range(4)]
    plans = [cio.Crc32Plan(offs, lens), cio.Crc32Plan(offs, lens)]
    s0 = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()
    K = 100
    for _ in range(10):
        plans[0].exec(bufs[0], outs[0], stream=s0)
    torch.cuda.synchronize()
    # 1. host cost per exec (queue only, no sync)
    t0 = time.perf_counter()
    for i in range(K):
        plans[0].exec(bufs[i % 4], outs[i % 4], stream=s0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host per exec {1e6 * (t1 - t0) / K:7.2f} us; wall per step single stream {1e6 * (t2 - t0) / K:7.2f} us")
    # 2. raw C launch loop: ctypes call with pre-built args
    import ctypes
    h = plans[0]._handle
    args = [(ctypes.c_void_p(bufs[i % 4].data_ptr()), ctypes.c_void_p(outs[i % 4].data_ptr())) for i in range(4)]
    sp = ctypes.c_void_p(int(s0.cuda_stream))
    fn = lib.cio_crc32_plan_exec
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        fn(h, args[i % 4][0], None, args[i % 4][1], sp)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"raw ctypes per exec {1e6 * (t1 - t0) / K:7.2f} us; wall per step {1e6 * (t2 - t0) / K:7.2f} us "
          f"= {total / ((t2 - t0) / K) / 1e9:8.1f} GB/s")
    # 3. two streams, two plans, alternating (independent batches overlap at kernel edges)
    sp1 = ctypes.c_void_p(int(s1.cuda_stream))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        fn(plans[i & 1]._handle, args[i % 4][0], None, args[i % 4][1], sp if (i & 1) == 0 else sp1)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"two streams wall per step {1e6 * (t2 - t0) / K:7.2f} us = {total / ((t2 - t0) / K) / 1e9:8.1f} GB/s")


if __name__ == "__main__":
    main()
