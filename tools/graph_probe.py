#!/usr/bin/env python3
"""Probe: cfg2 back-to-back launches on a stream vs the same launches replayed
from a captured HIP graph (4 rotating batches per graph).  Reports the mean
time per launch from one event pair around each timed region.

    python tools/graph_probe.py [--launches 400] [--rounds 4]
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
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--per-graph", type=int, default=4)
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
    plan = cio.Crc32Plan(offs, lens)
    s = torch.cuda.Stream(dev)
    ref = []
    with torch.cuda.stream(s):
        for b in range(nrot):
            plan.exec(bufs[b], outs[b], stream=s)
    torch.cuda.synchronize()
    ref = [o.clone() for o in outs]

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(a.per_graph):
            plan.exec(bufs[i % nrot], outs[i % nrot], stream=s)
    torch.cuda.synchronize()
    for o in outs:
        o.zero_()
    g.replay()
    torch.cuda.synchronize()
    same = all(torch.equal(ref[b], outs[b]) for b in range(min(nrot, a.per_graph)))
    print("graph replay outputs identical:", same, flush=True)

    def stream_run(n):
        with torch.cuda.stream(s):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for i in range(n):
                plan.exec(bufs[i % nrot], outs[i % nrot], stream=s)
            e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / n

    def graph_run(n):
        reps = n // a.per_graph
        with torch.cuda.stream(s):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(reps):
                g.replay()
            e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / (reps * a.per_graph)

    for _ in range(3):
        stream_run(200)
        graph_run(200)
    res = {"stream": [], "graph": []}
    for r in range(a.rounds):
        for k, fn in (("stream", stream_run), ("graph", graph_run)):
            us = fn(a.launches)
            res[k].append(us)
            print(f"round {r} {k:6s}: {us:7.2f} us/launch  {total / us / 1e3:7.1f} GB/s", flush=True)
    for k, v in res.items():
        print(f"{k}: median {np.median(v):.2f} us/launch, {total / np.median(v) / 1e3:.1f} GB/s")


if __name__ == "__main__":
    main()
