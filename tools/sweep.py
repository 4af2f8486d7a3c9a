#!/usr/bin/env python3
"""A/B sweep of kernel variants, interleaved in one process (guide rule 24).

    python tools/sweep.py [--iters 20] [--rounds 3] [--var CIO_GPU_RING=1,2,3] [--cfg cfg2,big]
    python tools/sweep.py --variants "CIO_GPU_THREADS=1024|CIO_GPU_THREADS=512,CIO_GPU_RING=2"

Each variant is a plan created with the given environment variables set (the
library reads tuning knobs at plan creation).  Every variant's output is
checked equal to the first variant's; per round and variant the mean kernel
time over `iters` launches (HIP events around the kernel) is printed, then the
median over rounds.
"""
import argparse
import json
import os
os.environ.setdefault("CIO_GPU_DIAG", "1")   # the library honours its A/B switches only with this
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--var", default="CIO_GPU_RING=1,2,3,4")
    ap.add_argument("--variants", default=None,
                    help="'|'-separated variants, each a comma-separated list of VAR=value")
    ap.add_argument("--cfg", default="cfg2,big")
    args = ap.parse_args()
    import torch
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl

    if args.variants:
        vals = args.variants.split("|")
        name = "variant"
    else:
        name, v = args.var.split("=")
        vals = [f"{name}={x}" for x in v.split(",")]

    def apply(v):
        for kv in v.split(","):
            k, x = kv.split("=")
            os.environ[k] = x

    def clear(v):
        for kv in v.split(","):
            os.environ.pop(kv.split("=")[0], None)
    dev = torch.device("cuda:0")
    lib = cio.lib()
    results = {}
    for cfg in args.cfg.split(","):
        if cfg == "cfg2":
            lens = wl.cfg2_lens()
        elif cfg == "big":
            lens = np.full(1024, 4 * 1024 * 1024, np.uint64)
        elif cfg == "cfg3":
            lens = wl.cfg3_lens()
        elif cfg == "small":
            lens = np.full(65536, 4096, np.uint64)
        else:
            raise ValueError(cfg)
        offs = wl.packed_offsets(lens, align=16)
        total = wl.batch_bytes(offs, lens)
        nrot = max(2, min(4, int(1.2e9 // max(total, 1)) + 1))
        bufs = []
        for b in range(nrot):
            t = torch.empty(total + 64, dtype=torch.uint8, device=dev)
            cio.fill_synthetic(t, offs, lens, 0xC0DE + b)
            bufs.append(t)
        out = torch.empty(len(lens), dtype=torch.int32, device=dev)
        plans = {}
        for v in vals:
            apply(v)
            plans[v] = cio.Crc32Plan(offs, lens)
            clear(v)
        ref = None
        for v in vals:
            plans[v].exec(bufs[0], out)
            torch.cuda.synchronize()
            got = out.cpu().numpy().copy()
            if ref is None:
                ref = got
            assert np.array_equal(got, ref), f"variant {v} differs"
        times = {v: [] for v in vals}
        evs = [(lib.cio_gpu_event_create(), lib.cio_gpu_event_create()) for _ in range(args.iters)]
        for r in range(args.rounds):
            for v in vals:
                for i in range(3):
                    plans[v].exec(bufs[i % nrot], out)
                for i in range(args.iters):
                    plans[v].exec_events(bufs[i % nrot], out, evs[i][0], evs[i][1])
                torch.cuda.synchronize()
                ms = float(np.mean([lib.cio_gpu_event_elapsed_ms(a, b) for a, b in evs]))
                times[v].append(ms * 1e3)
                print(f"{cfg} round {r} {v}: {ms * 1e3:8.2f} us  {total / ms / 1e6:8.1f} GB/s",
                      flush=True)
        for v in vals:
            med = float(np.median(times[v]))
            results[f"{cfg}/{v}"] = {"us": round(med, 2), "GBps": round(total / med / 1e3, 1)}
        for p in plans.values():
            p.close()
        del bufs
        torch.cuda.empty_cache()
    print(json.dumps(results))


if __name__ == "__main__":
    main()
