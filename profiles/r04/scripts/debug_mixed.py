#!/usr/bin/env python3
"""Diagnostic: GPU batch CRC of a mixed-size batch vs the C oracle, under
several plan environments (e.g. CIO_GPU_TAIL=0 vs default), repeated launches.

    python tools/debug_mixed.py [n_chunks] [launches]
"""
import os
os.environ.setdefault("CIO_GPU_DIAG", "1")   # the library honours its A/B switches only with this
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    import torch
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl
    from oracle import pyoracle as po
    dev = torch.device("cuda:0")
    lens = wl.cfg3_lens(n)
    offs = wl.packed_offsets(lens)
    total = wl.batch_bytes(offs, lens)
    buf = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    cio.fill_synthetic(buf, offs, lens, 0x1234)
    host = buf.cpu().numpy()
    want = po.crc_batch(host, offs, lens)
    print(f"n={n} bytes={total / 1e9:.2f} GB", flush=True)
    for env in (os.environ.get("DEBUG_ENVS") or "CIO_GPU_TAIL=0|").split("|"):
        saved = {}
        for kv in filter(None, env.split(",")):
            k, v = kv.split("=")
            saved[k] = os.environ.get(k)
            os.environ[k] = v
        plan = cio.Crc32Plan(offs, lens)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
        out = torch.empty(n, dtype=torch.int32, device=dev)
        for it in range(launches):
            plan.exec(buf, out)
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            bad = np.nonzero(got != want)[0]
            print(f"env[{env or 'default'}] launch {it}: mismatches {len(bad)} first {bad[:8].tolist()}", flush=True)
        plan.close()


if __name__ == "__main__":
    main()
