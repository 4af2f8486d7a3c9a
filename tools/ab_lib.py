#!/usr/bin/env python3
"""In-process A/B of two builds of libchunkio_amd.so (guide rule 24).

    python tools/ab_lib.py --libs chunkio_amd/lib/ab/prev.so,chunkio_amd/lib/libchunkio_amd.so \
        [--cfg cfg2,big] [--iters 20] [--rounds 3] [--env "CIO_GPU_DYN=0|CIO_GPU_DYN=0"]

Each library gets its own plan over the same device buffers; outputs must be
identical; rounds interleave the libraries so clock/thermal drift hits both.
`--env` optionally gives per-library plan-creation environment ('|'-separated).
"""
import argparse
import ctypes
import json
import time
import os
os.environ.setdefault("CIO_GPU_DIAG", "1")   # the library honours its A/B switches only with this
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

U64P = ctypes.POINTER(ctypes.c_uint64)


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    lib.cio_crc32_plan_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), U64P, U64P, ctypes.c_size_t]
    lib.cio_crc32_plan_exec.argtypes = [ctypes.c_void_p] * 5
    lib.cio_crc32_plan_exec_events.argtypes = [ctypes.c_void_p] * 7
    lib.cio_crc32_plan_destroy.argtypes = [ctypes.c_void_p]
    lib.cio_gpu_event_create.restype = ctypes.c_void_p
    lib.cio_gpu_event_elapsed_ms.restype = ctypes.c_float
    lib.cio_gpu_event_elapsed_ms.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.cio_gpu_event_record.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.cio_gpu_event_destroy.argtypes = [ctypes.c_void_p]
    lib.cio_gpu_version.restype = ctypes.c_char_p
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--env", default=None)
    ap.add_argument("--cfg", default="cfg2,big")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--warm-s", type=float, default=1.0, help="untimed launches before each batch's rounds")
    ap.add_argument("--no-check", action="store_true", help="ablation builds: skip the output equality check")
    args = ap.parse_args()
    import torch
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl

    paths = args.libs.split(",")
    envs = args.env.split("|") if args.env else [""] * len(paths)
    libs = [load(p) for p in paths]
    for p, lib in zip(paths, libs):
        print(f"{p}: {lib.cio_gpu_version().decode()}", flush=True)
        if hasattr(lib, "cioa_debug_dispatch_delays"):
            d = (ctypes.c_float * 8)()
            lib.cioa_debug_dispatch_delays(d)
            print("   dispatch delays us by blockIdx%8:", " ".join(f"{x:.2f}" for x in d), flush=True)
    dev = torch.device("cuda:0")
    results = {}
    for cfg in args.cfg.split(","):
        k4n, klen = 0, 4096
        if cfg.startswith("k4x"):       # k4x<n>: n chunks of 4 KiB
            k4n = int(cfg[3:])
        elif cfg.startswith("c") and "kx" in cfg:   # c<K>kx<n>: n chunks of K KiB
            klen, k4n = int(cfg[1:cfg.index("kx")]) << 10, int(cfg[cfg.index("kx") + 2:])
        lens = (lambda: np.full(k4n, klen, np.uint64)) if k4n else {
                "cfg2": wl.cfg2_lens, "cfg3": wl.cfg3_lens,
                "big": lambda: np.full(1024, 4 << 20, np.uint64),
                "cfg4": lambda: np.full(8192, 4 << 20, np.uint64),
                "mid": lambda: np.full(1024, 1638400, np.uint64),
                "small": lambda: np.full(65536, 4096, np.uint64),
                "cfg4k": lambda: np.full(102400, 4096, np.uint64)}[cfg]
        lens = lens()
        assert len(lens) > 0, cfg
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        offs = np.ascontiguousarray(wl.packed_offsets(lens, align=16), dtype=np.uint64)
        total = int(wl.batch_bytes(offs, lens))
        nrot = max(2, min(4, int(1.2e9 // max(total, 1)) + 1))
        bufs = []
        for b in range(nrot):
            t = torch.empty(total + 64, dtype=torch.uint8, device=dev)
            cio.fill_synthetic(t, offs, lens, 0xC0DE + b)
            bufs.append(t)
        outs = [torch.empty(len(lens), dtype=torch.int32, device=dev) for _ in libs]
        plans = []
        for lib, env in zip(libs, envs):
            saved = {}
            for kv in filter(None, env.split(",")):
                k, v = kv.split("=")
                saved[k] = os.environ.get(k)
                os.environ[k] = v
            p = ctypes.c_void_p()
            rc = lib.cio_crc32_plan_create(ctypes.byref(p), offs.ctypes.data_as(U64P),
                                           lens.ctypes.data_as(U64P), len(lens))
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k)
                else:
                    os.environ[k] = v
            assert rc == 0, "plan_create failed"
            plans.append(p)
        stream = torch.cuda.current_stream().cuda_stream
        ref = None
        for lib, p, o in zip(libs, plans, outs):
            assert lib.cio_crc32_plan_exec(p, bufs[0].data_ptr(), None, o.data_ptr(), stream) == 0
            torch.cuda.synchronize()
            got = o.cpu().numpy().copy()
            ref = got if ref is None else ref
            assert args.no_check or np.array_equal(got, ref), f"{cfg}: outputs differ"
        times = [[] for _ in libs]
        times_b2b = [[] for _ in libs]
        # Warm the clocks first: short A/Bs on a cold GPU drift faster round
        # by round (profiles/r05/camping/), which biases the later libs.
        t_end = time.perf_counter() + args.warm_s
        while time.perf_counter() < t_end:
            for k in range(8):
                libs[0].cio_crc32_plan_exec(plans[0], bufs[k % nrot].data_ptr(), None, outs[0].data_ptr(), stream)
            torch.cuda.synchronize()
        order = list(range(len(libs)))
        # one set of events per lib for the whole batch, destroyed after it
        all_evs = [[(lib.cio_gpu_event_create(), lib.cio_gpu_event_create()) for _ in range(args.iters)]
                   for lib in libs]
        all_b2b = [(lib.cio_gpu_event_create(), lib.cio_gpu_event_create()) for lib in libs]
        assert all(e for evs in all_evs for pair in evs for e in pair) and all(e for pr in all_b2b for e in pr)
        for r in range(args.rounds):
            # ABBA: odd rounds run the libs in reverse order
            for i in (order if r % 2 == 0 else order[::-1]):
                lib, p, o = libs[i], plans[i], outs[i]
                evs = all_evs[i]
                for k in range(3):
                    lib.cio_crc32_plan_exec(p, bufs[k % nrot].data_ptr(), None, o.data_ptr(), stream)
                for k in range(args.iters):
                    lib.cio_crc32_plan_exec_events(p, bufs[k % nrot].data_ptr(), None, o.data_ptr(),
                                                   stream, evs[k][0], evs[k][1])
                torch.cuda.synchronize()
                ms = [lib.cio_gpu_event_elapsed_ms(a, b) for a, b in evs]
                assert min(ms) > 0, f"{cfg}: event timing failed"
                us = float(np.mean(ms)) * 1e3
                # back-to-back launches under one event pair (no per-launch events)
                b0, b1 = all_b2b[i]
                lib.cio_gpu_event_record(b0, stream)
                for k in range(args.iters):
                    lib.cio_crc32_plan_exec(p, bufs[k % nrot].data_ptr(), None, o.data_ptr(), stream)
                lib.cio_gpu_event_record(b1, stream)
                torch.cuda.synchronize()
                us_b2b = lib.cio_gpu_event_elapsed_ms(b0, b1) * 1e3 / args.iters
                times[i].append(us)
                times_b2b[i].append(us_b2b)
                print(f"{cfg} round {r} lib{i}: {us:8.2f} us  {total / us / 1e3:8.1f} GB/s   "
                      f"back-to-back {us_b2b:8.2f} us/launch", flush=True)
        for i in range(len(libs)):
            med = float(np.median(times[i]))
            results[f"{cfg}/lib{i}"] = {"us": round(med, 2), "GBps": round(total / med / 1e3, 1),
                                        "b2b_us": round(float(np.median(times_b2b[i])), 2)}
        for lib, p, evs, pr in zip(libs, plans, all_evs, all_b2b):
            lib.cio_crc32_plan_destroy(p)
            for e in [x for pair in evs for x in pair] + list(pr):
                lib.cio_gpu_event_destroy(e)
        del bufs
        torch.cuda.empty_cache()
    print(json.dumps(results))


if __name__ == "__main__":
    main()
