#!/usr/bin/env python3
"""Read-only stream with intra-workgroup balancing (CIO_GPU_RS_WGPOOL=k: the
last k steps of each wave's range pooled per workgroup, claimed through an
LDS atomic) against the static split, interleaved rounds in one process.

    python tools/rs_pool_probe.py [--cfg cfg2] [--ks 0,1,2,4] [--rounds 4] [--iters 50]
"""
import argparse
import os
os.environ.setdefault("CIO_GPU_DIAG", "1")   # the library honours its A/B switches only with this
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="cfg2")
    ap.add_argument("--ks", default="0,1,2,4")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    import torch
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl
    lens = wl.cfg2_lens() if args.cfg == "cfg2" else np.full(1024, 4 << 20, np.uint64)
    offs = wl.packed_offsets(lens, align=16)
    total = int(wl.batch_bytes(offs, lens))
    dev = torch.device("cuda:0")
    bufs = [torch.empty(total + 64, dtype=torch.uint8, device=dev) for _ in range(4)]
    for b, t in enumerate(bufs):
        cio.fill_synthetic(t, offs, lens, 7 + b)
    lib = cio.lib()
    s = torch.cuda.current_stream().cuda_stream
    ks = [int(x) for x in args.ks.split(",")]
    res = {k: [] for k in ks}
    for r in range(args.rounds):
        for k in ks:
            if k:
                os.environ["CIO_GPU_RS_WGPOOL"] = str(k)
            else:
                os.environ.pop("CIO_GPU_RS_WGPOOL", None)
            for i in range(10):
                lib.cio_gpu_read_stream(bufs[i % 4].data_ptr(), total, s)
            e0, e1 = lib.cio_gpu_event_create(), lib.cio_gpu_event_create()
            lib.cio_gpu_event_record(e0, s)
            for i in range(args.iters):
                lib.cio_gpu_read_stream(bufs[i % 4].data_ptr(), total, s)
            lib.cio_gpu_event_record(e1, s)
            torch.cuda.synchronize()
            us = lib.cio_gpu_event_elapsed_ms(e0, e1) * 1e3 / args.iters
            res[k].append(us)
            print(f"round {r} pool k={k}: {us:8.2f} us/launch  {total / us / 1e3:8.1f} GB/s", flush=True)
    for k in ks:
        print(f"k={k}: median {np.median(res[k]):8.2f} us  {res[k]}")


if __name__ == "__main__":
    main()
