#!/usr/bin/env python3
"""Latency of ONE chunk's CRC: the GPU host batch against the library's host
crc_update, region sizes 16 B .. 8 MiB.

    python tools/crossover.py [out.txt]

For each size: the median wall time of
  - crc_update(init, buf, n)                  (crc32_host.c, calling thread)
  - cio_crc32_batch_host(&buf, &n, ..., 1)     (pinned staging + H2D + kernel
                                                + D2H, synchronous)
over a buffer that stays in host cache between calls, as a chunk's mapped
page does in the chunk layer's single-chunk paths (cioa_chunk.c: verify on
open/up, recompute, deferred catch-up).  Also times the reference tests'
down/up loop (tests/fs.c issue_flb_2025: 1000 down/up cycles of a 20-byte
chunk) in the C replay with every CRC on the GPU (CIOA_CPU_CRC_MAX=0) and
with the library's default routing.  Prints a table and the crossover.
"""
import ctypes
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def median_time(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    import chunkio_amd as cio
    lib = cio.lib()
    rng = np.random.default_rng(5)
    sizes = [16, 64, 256, 1024, 4096, 16384, 65536, 131072, 262144, 524288, 1 << 20, 2 << 20, 4 << 20, 8 << 20]
    lines = ["size_B  cpu_crc_update_us  gpu_one_chunk_us  cpu_GBps  gpu_GBps  faster"]
    rows = []
    out = np.zeros(1, np.uint32)
    for n in sizes:
        buf = rng.integers(0, 256, n, dtype=np.uint8)
        ptr = ctypes.c_void_p(buf.ctypes.data)
        ptrs = (ctypes.c_void_p * 1)(buf.ctypes.data)
        lens = (ctypes.c_size_t * 1)(n)
        op = out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))

        def cpu():
            lib.crc_update(0xFFFFFFFF, ptr, n)

        def gpu():
            if lib.cio_crc32_batch_host(ptrs, lens, None, op, 1) != 0:
                raise RuntimeError(lib.cio_gpu_last_error())

        for _ in range(20):
            gpu()
            cpu()
        reps = 400 if n <= (1 << 20) else 100
        tc = median_time(cpu, reps)
        tg = median_time(gpu, reps)
        want = int(lib.crc_update(0xFFFFFFFF, ptr, n)) & 0xFFFFFFFF
        gpu()
        assert int(out[0]) == want, (n, hex(int(out[0])), hex(want))
        rows.append((n, tc, tg))
        lines.append(f"{n:>8}  {tc * 1e6:>17.2f}  {tg * 1e6:>16.2f}  {n / tc / 1e9:>8.2f}  {n / tg / 1e9:>8.2f}  "
                     f"{'cpu' if tc < tg else 'gpu'}")
    cross = None
    for n, tc, tg in rows:
        if tg < tc:
            cross = n
            break
    last_cpu = max([n for n, tc, tg in rows if tc <= tg] or [0])
    lines.append(f"first size where the GPU round trip wins: {cross} B; largest size where the host "
                 f"crc_update wins: {last_cpu} B; library default cio_crc32_cpu_max() = {lib.cio_crc32_cpu_max()} B")

    # tests/fs.c issue_flb_2025 through the C replay: GPU route vs default routing
    binp = os.path.join(ROOT, "tests", "c", "bin", "test_chunk_api")
    data = os.path.join(ROOT, "tests", "golden", "400kb.txt")
    if os.path.exists(binp):
        import tempfile
        for label, env in (("all-GPU (CIOA_CPU_CRC_MAX=0)", {"CIOA_CPU_CRC_MAX": "0"}),
                           ("default routing", {})):
            with tempfile.TemporaryDirectory() as tmp:
                e = {k: v for k, v in os.environ.items() if k != "CIOA_CPU_CRC_MAX"}
                e.update(env)
                t0 = time.perf_counter()
                r = subprocess.run([binp, data, tmp, "immediate", "issue_flb_2025"], env=e,
                                   capture_output=True, text=True, timeout=600)
                dt = time.perf_counter() - t0
                ok = r.returncode == 0 and "0 failed" in r.stdout
            lines.append(f"issue_flb_2025 (1000 down/up cycles), {label}: {dt * 1e3:.1f} ms wall, ok={ok}")
            t0 = time.perf_counter()
    text = "\n".join(lines)
    print(text, flush=True)
    if out_path:
        with open(out_path, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
