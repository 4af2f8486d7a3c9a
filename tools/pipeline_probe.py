#!/usr/bin/env python3
"""Probe: cfg2 batches launched back to back on one stream vs alternated over
two streams (one plan each), interleaved over several rounds in one process.
Reports the mean time per batch from one event pair around each timed region.

    python tools/pipeline_probe.py [--launches 400] [--rounds 6]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=6)
    a = ap.parse_args()
    import torch
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl
    dev = torch.device("cuda:0")
    lens = np.full(wl.CFG2_N, wl.CFG2_LEN, dtype=np.uint64)
    offs = wl.packed_offsets(lens, align=16)
    total = wl.batch_bytes(offs, lens)
    nrot = 4
    bufs, outs = [], []
    for b in range(nrot):
        t = torch.empty(total + 64, dtype=torch.uint8, device=dev)
        cio.fill_synthetic(t, offs, lens, wl.CFG2_SEED + b)
        bufs.append(t)
        outs.append(torch.empty(len(lens), dtype=torch.int32, device=dev))
    plans = [cio.Crc32Plan(offs, lens), cio.Crc32Plan(offs, lens)]
    s1 = torch.cuda.current_stream(dev)
    s2 = torch.cuda.Stream(dev)

    def run(n, two):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s1)
        s2.wait_stream(s1)
        for i in range(n):
            k = (i & 1) if two else 0
            plans[k].exec(bufs[i % nrot], outs[i % nrot], stream=(s1, s2)[k])
        s1.wait_stream(s2)
        e1.record(s1)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / n

    for _ in range(5):
        run(200, False)
        run(200, True)
    res = {"one stream": [], "two streams": []}
    for r in range(a.rounds):
        for k, two in (("one stream", False), ("two streams", True)):
            us = run(a.launches, two)
            res[k].append(us)
            print(f"round {r} {k:11s}: {us:7.2f} us/batch  {total / us / 1e3:7.1f} GB/s", flush=True)
    for k, v in res.items():
        print(f"{k}: median {np.median(v):.2f} us/batch, {total / np.median(v) / 1e3:.1f} GB/s")


if __name__ == "__main__":
    main()
