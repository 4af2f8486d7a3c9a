"""Host-side ceilings of the verify-on-load leg, no GPU work: how fast can T
threads move 1000 chunk files (page cache) into pinned memory, by pread()
and by mmap + memcpy?  Used to locate the bound of cio_verify_paths
(DESIGN.md §4a).

    python tools/host_read_probe.py [threads ...]
"""
import mmap
import os
import shutil
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    threads = [int(a) for a in sys.argv[1:]] or [8, 16, 32]
    d400 = np.fromfile(os.path.join(ROOT, "tests", "golden", "400kb.txt"), dtype=np.uint8)
    blob = np.tile(d400, 5)
    root = tempfile.mkdtemp(prefix="cioa-readprobe-")
    try:
        paths = []
        for i in range(1000):
            p = os.path.join(root, f"f{i:04d}")
            blob.tofile(p)
            paths.append(p)
        size = blob.size
        pinned = torch.empty(len(paths) * size, dtype=torch.uint8).pin_memory()
        dst = pinned.numpy()
        fds = [os.open(p, os.O_RDONLY) for p in paths]
        for T in threads:
            def rd(k):
                for i in range(k, len(fds), T):
                    os.preadv(fds[i], [memoryview(dst[i * size:(i + 1) * size])], 0)

            def mm(k):
                for i in range(k, len(fds), T):
                    m = mmap.mmap(fds[i], size, prot=mmap.PROT_READ)
                    dst[i * size:(i + 1) * size] = np.frombuffer(m, np.uint8)
                    m.close()
            for name, fn in (("pread", rd), ("mmap_memcpy", mm)):
                best = 1e9
                with ThreadPoolExecutor(T) as ex:
                    for _ in range(4):
                        t0 = time.perf_counter()
                        list(ex.map(fn, range(T)))
                        best = min(best, time.perf_counter() - t0)
                print(f"threads={T:3d} {name:12s} {len(paths) * size / best / 1e9:7.1f} GB/s", flush=True)
        for fd in fds:
            os.close(fd)
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
