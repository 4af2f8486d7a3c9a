#!/usr/bin/env python3
"""Read-only stream vs bytes per lane per load group (diagnostic,
CIO_GPU_RS_LANE=16|32|64): coalesced 1 KiB rows against 32- or 64-byte
contiguous runs per lane, on rotating cfg2 buffers, the CRC kernel's split."""
import os
os.environ.setdefault("CIO_GPU_DIAG", "1")   # the library honours its A/B switches only with this
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl
    lanes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "16,32,64").split(",")]
    lens = wl.cfg2_lens()
    offs = wl.packed_offsets(lens, align=16)
    total = int(wl.batch_bytes(offs, lens))
    bufs = [torch.empty(total + 64, dtype=torch.uint8, device="cuda") for _ in range(4)]
    for b, t in enumerate(bufs):
        cio.fill_synthetic(t, offs, lens, 1 + b)
    lib = cio.lib()
    s = torch.cuda.current_stream().cuda_stream
    for rnd in range(4):
        for lb in lanes:
            os.environ["CIO_GPU_RS_LANE"] = str(lb)
            for i in range(20):
                lib.cio_gpu_read_stream(bufs[i % 4].data_ptr(), total, s)
            e0, e1 = lib.cio_gpu_event_create(), lib.cio_gpu_event_create()
            lib.cio_gpu_event_record(e0, s)
            n = 100
            for i in range(n):
                lib.cio_gpu_read_stream(bufs[i % 4].data_ptr(), total, s)
            lib.cio_gpu_event_record(e1, s)
            torch.cuda.synchronize()
            ms = lib.cio_gpu_event_elapsed_ms(e0, e1) / n
            print(f"round {rnd} lane bytes {lb:2d}: {ms * 1e3:7.2f} us  {total / (ms * 1e-3) / 1e9:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
