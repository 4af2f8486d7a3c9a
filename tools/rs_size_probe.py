#!/usr/bin/env python3
"""Does the per-wave range size matter to HBM?  The read-only stream
(read_stream_kernel: the CRC kernels' even split of 4 KiB steps over 4096
waves, contiguous range per wave) over batches of w steps per wave, w around
powers of two: at w = 2^k every wave's range starts at an address congruent
modulo 2^k x 4 KiB, so at any moment all waves read lines with the same low
address bits.  GB/s per w, 4 rotating buffers, 3 rounds interleaved.

    python tools/rs_size_probe.py [w,w,...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import chunkio_amd as cio
    ws = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else
                           "16,17,24,25,31,32,33,48,50,63,64,65,96,100,127,128,129").split(",")]
    grids = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "256").split(",")]
    lib = cio.lib()
    s = torch.cuda.current_stream().cuda_stream
    W = 4096
    res = {(w, g): [] for w in ws for g in grids}
    maxb = max(ws) * W * 4096
    bufs = [torch.empty(maxb, dtype=torch.uint8, device="cuda") for _ in range(4)]
    for b in bufs:
        b.fill_(7)
    for rnd in range(3):
        for w in ws:
            for g in grids:
                total = w * W * 4096       # w steps per wave on the full 256-workgroup grid
                for i in range(8):
                    lib.cio_gpu_read_stream_grid(bufs[i % 4].data_ptr(), total, g, s)
                e0, e1 = lib.cio_gpu_event_create(), lib.cio_gpu_event_create()
                n = max(10, 2000 // w)
                lib.cio_gpu_event_record(e0, s)
                for i in range(n):
                    lib.cio_gpu_read_stream_grid(bufs[i % 4].data_ptr(), total, g, s)
                lib.cio_gpu_event_record(e1, s)
                torch.cuda.synchronize()
                ms = lib.cio_gpu_event_elapsed_ms(e0, e1) / n
                res[(w, g)].append(total / (ms * 1e-3) / 1e9)
                lib.cio_gpu_event_destroy(e0)
                lib.cio_gpu_event_destroy(e1)
        print(f"round {rnd}: " + " ".join(f"{w}/{g}:{res[(w, g)][-1]:.0f}" for w in ws for g in grids), flush=True)
    print("\nsteps/wave (256 WGs)  MiB/wave  " + "  ".join(f"GB/s grid {g}" for g in grids) + "  (best of 3)")
    for w in ws:
        print(f"{w:9d}  {w * 4096 / 2**20:8.3f}  " + "  ".join(f"{max(res[(w, g)]):12.1f}" for g in grids))


if __name__ == "__main__":
    main()
