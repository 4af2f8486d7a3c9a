#!/usr/bin/env python3
"""Verify-on-load of 1000 perf-test chunk files (2 MB each, page cache) by one
cio_verify_paths call per route setting, interleaved over rounds: the host
alone, the GPU alone, and the default route (the split route, rates learned
over the calls) at several host thread counts.  Prints GB/s per setting (min time per round,
median over rounds) and checks that every setting returns the same results.

    python tools/split_probe.py [rounds]
"""
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    import chunkio_amd as cio
    if os.environ.get("SPLIT_PROBE_BIND") == "1":
        # as bench.py's host legs do: this process on the GPU's NUMA node
        import bench
        print("bound to", bench.bind_to_gpu_node(0), "CPUs", flush=True)
    from chunkio_amd import chunkfile as cf
    d400 = np.fromfile(os.path.join(ROOT, "tests", "golden", "400kb.txt"), dtype=np.uint8).tobytes()
    root = tempfile.mkdtemp(prefix="cioa-split-")
    files = 1000
    try:
        paths = [os.path.join(root, "s", f"perf-test-{i:04d}.txt") for i in range(files)]
        c, _ = cf.ChunkFile.open(paths[0])
        for _ in range(5):
            c.write(d400)
        c.sync()
        c.close()
        for p in paths[1:]:
            shutil.copyfile(paths[0], p)
        region = files * (2 + 5 * len(d400))
        settings = [("host T=1", dict(cpu_max=-1, threads=1), "0"),
                    ("gpu alone", dict(threads=1, split=False), "0"),
                    ("default T=1 (split)", dict(threads=1), "0"),
                    ("host T=4", dict(cpu_max=-1, threads=4), "0"),
                    ("default T=4 (split)", dict(threads=4), "0"),
                    ("host T=8", dict(cpu_max=-1, threads=8), "0"),
                    ("default T=8 (split)", dict(threads=8), "0"),
                    ("host T=16", dict(cpu_max=-1, threads=16), "0"),
                    ("default T=16 (split)", dict(threads=16), "0")]
        res = {name: [] for name, _, _ in settings}
        ref = None
        for r in range(rounds):
            order = settings if r % 2 == 0 else settings[::-1]
            for name, kw, hf in order:
                cio.route(reset=True, **kw)
                out = cf.verify_paths(paths)
                ts = []
                for _ in range(3):
                    t0 = time.perf_counter()
                    out = cf.verify_paths(paths)
                    ts.append(time.perf_counter() - t0)
                if ref is None:
                    ref = out
                assert all(np.array_equal(a, b) for a, b in zip(out, ref)), name
                res[name].append(region / min(ts) / 1e9)
            print(f"round {r}: " + "  ".join(f"{n} {res[n][-1]:.1f}" for n, _, _ in settings), flush=True)
        cio.route(reset=True)
        print("learned split rates (T = 16):", cio.split_rates())
        print("\nGB/s (median of rounds, best of 3 calls each):")
        for n, _, _ in settings:
            print(f"  {n:24s} {np.median(res[n]):7.1f}   [{min(res[n]):.1f} .. {max(res[n]):.1f}]")
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
