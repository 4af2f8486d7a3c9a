#!/usr/bin/env python3
"""Per-wave timestamps of the read-only stream kernel on the cfg2 batch
(CIO_GPU_RS_STAMPS=1), printed like tools/stamps.py prints the CRC kernel's:
does the read-only kernel have the CRC kernel's spread of per-wave finish
times, or is that spread the CRC's own?"""
import ctypes
import os
os.environ.setdefault("CIO_GPU_DIAG", "1")   # the library honours its A/B switches only with this
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    os.environ["CIO_GPU_RS_STAMPS"] = "1"
    import torch
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl
    lens = wl.cfg2_lens()
    offs = wl.packed_offsets(lens, align=16)
    total = int(wl.batch_bytes(offs, lens))
    bufs = []
    for b in range(4):
        bufs.append(torch.empty(total + 64, dtype=torch.uint8, device="cuda"))
        cio.fill_synthetic(bufs[-1], offs, lens, 1 + b)
    lib = cio.lib()
    f = lib.cioa_debug_rs_stamps
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t]
    s = torch.cuda.current_stream().cuda_stream
    q = lambda a: " ".join(f"{np.percentile(a, p):7.2f}" for p in (0, 10, 50, 90, 100))  # noqa: E731
    for it in range(5):
        for k in range(16):
            lib.cio_gpu_read_stream(bufs[(it + k) % 4].data_ptr(), total, s)
        torch.cuda.synchronize()
        st = np.zeros(4096 * 4 * 2, np.uint64)
        W = f(st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), st.size)
        raw = st[:W * 4].reshape(W, 4).astype(np.int64)
        t0 = raw[:, 0].min()
        us = (raw[:, :3] - t0) / 100.0
        print(f"read-only cfg2 iter {it}: span {us[:, 2].max():7.2f} us   [pct 0/10/50/90/100]")
        print("   entry      ", q(us[:, 0]))
        print("   first step ", q(us[:, 1]))
        print("   stream done", q(us[:, 2]))
        print("   stream dur ", q(us[:, 2] - us[:, 1]))
        wg = us[:, 2].reshape(-1, 16)
        print("   WG max done", q(wg.max(1)))
        print("   WG spread  ", q(wg.max(1) - wg.min(1)))
        xcd = np.arange(wg.shape[0]) % 8
        print("   WG max by blockIdx%8   ", " ".join(f"{wg.max(1)[xcd == k].mean():6.1f}" for k in range(8)))


if __name__ == "__main__":
    main()
