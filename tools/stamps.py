#!/usr/bin/env python3
"""Per-wave phase timestamps of the CRC kernel (diagnostic build, CIO_GPU_STAMPS=1)."""
import ctypes
import os
os.environ.setdefault("CIO_GPU_DIAG", "1")   # the library honours its A/B switches only with this
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    os.environ["CIO_GPU_STAMPS"] = "1"
    import torch
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    tag = sys.argv[2] if len(sys.argv) > 2 else cfg
    lens = wl.cfg2_lens() if cfg == "cfg2" else np.full(1024, 4 << 20, np.uint64)
    offs = wl.packed_offsets(lens, align=16)
    dev = torch.device("cuda:0")
    # Rotate 4 batches like bench.py, so the 256 MiB Infinity Cache cannot
    # serve a launch from the previous one.
    bufs = []
    for b in range(4):
        bufs.append(torch.empty(wl.batch_bytes(offs, lens) + 64, dtype=torch.uint8, device=dev))
        cio.fill_synthetic(bufs[-1], offs, lens, 1 + b)
    out = torch.empty(len(lens), dtype=torch.int32, device=dev)
    plan = cio.Crc32Plan(offs, lens)
    f = cio.lib().cioa_debug_stamps
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t]
    for it in range(5):
        # 16 back-to-back launches (warm clocks, rotating batches); the stamps
        # are those of the last one.
        for k in range(16):
            plan.exec(bufs[(it + k) % 4], out)
        torch.cuda.synchronize()
        K = 16                    # kStampWords (cio_gpu_internal.h)
        st = np.zeros(4096 * K * 2, np.uint64)
        W = f(plan._handle, st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), st.size)
        raw = st[:W * K].reshape(W, K).astype(np.int64)
        # entry, tables, stream, exit, first, mid, loads issued, build phase 1, build phase 2, step 1,
        # arrived, barrier 1, barrier 2, folded
        t = np.concatenate([raw[:, :4], raw[:, 6:16]], axis=1)
        hw, xcc = raw[:, 4], raw[:, 5]
        simd = (hw >> 4) & 3
        print("   simd of wave slot (WG 0..3):", [list(simd.reshape(-1, 16)[b]) for b in range(4)])
        print("   xcc of WG 0..15:", list((xcc.reshape(-1, 16)[:, 0] & 0xf)[:16]))
        t0 = t[:, 0].min()
        us = (t - t0) / 100.0     # 100 MHz
        q = lambda a: " ".join(f"{np.percentile(a, p):7.2f}" for p in (0, 10, 50, 90, 100))  # noqa: E731
        print(f"{cfg} iter {it}: span {us[:, 3].max():7.2f} us   [pct 0/10/50/90/100]")
        print("   entry      ", q(us[:, 0]))
        print("   loads issued", q(us[:, 6]))
        print("   build ph1   ", q(us[:, 7]))
        print("   build ph2   ", q(us[:, 8]))
        print("   tables done", q(us[:, 1]))
        print("   first step ", q(us[:, 4]))
        print("   first-tabl ", q(us[:, 4] - us[:, 1]))
        print("   step 1 done", q(us[:, 9]))
        print("   mid step   ", q(us[:, 5]))
        print("   1st half   ", q(us[:, 5] - us[:, 4]), " 2nd half", q(us[:, 2] - us[:, 5]))
        print("   stream done", q(us[:, 2]))
        print("   exit       ", q(us[:, 3]))
        print("   stream dur ", q(us[:, 2] - us[:, 1]))
        print("   tail dur   ", q(us[:, 3] - us[:, 2]))
        print("   arrived - stream done ", q(us[:, 10] - us[:, 2]))
        print("   barrier1 - arrived    ", q(us[:, 11] - us[:, 10]))
        print("   barrier2 - barrier1   ", q(us[:, 12] - us[:, 11]))
        print("   folded - barrier2     ", q(us[:, 13] - us[:, 12]))
        print("   exit - folded         ", q(us[:, 3] - us[:, 13]))
        wgb1 = us[:, 11].reshape(-1, 16)
        print("   WG barrier1 - WG max stream done", q(wgb1.max(1) - us[:, 2].reshape(-1, 16).max(1)))
        lastw = int(np.argmax(us[:, 3]))
        print("   last wave: stream %.2f arrived %.2f bar1 %.2f bar2 %.2f folded %.2f exit %.2f" %
              tuple(us[lastw, k] for k in (2, 10, 11, 12, 13, 3)))
        ent = us[:, 0].reshape(-1, 16)
        tab = us[:, 1].reshape(-1, 16)
        print("   WG entry spread (last-first wave)", q(ent.max(1) - ent.min(1)))
        print("   WG first entry                   ", q(ent.min(1)))
        print("   WG tables - last entry           ", q(tab.max(1) - ent.max(1)))
        iss = us[:, 6].reshape(-1, 16)
        bld = us[:, 7].reshape(-1, 16)
        print("   WG issued spread (last-first)    ", q(iss.max(1) - iss.min(1)))
        print("   WG build spread (last-first)     ", q(bld.max(1) - bld.min(1)))
        print("   WG tables - WG last build        ", q(tab.max(1) - bld.max(1)))
        print("   WG tables - WG first build       ", q(tab.max(1) - bld.min(1)))
        print("   issued - entry by wave slot", " ".join(f"{x:5.2f}" for x in (iss - ent).mean(0)))
        wg = us[:, 2].reshape(-1, 16)
        print("   WG max done", q(wg.max(1)))
        print("   WG min done", q(wg.min(1)))
        print("   WG spread  ", q(wg.max(1) - wg.min(1)))
        ex = us[:, 3].reshape(-1, 16)
        print("   WG exit - WG max done", q(ex.max(1) - wg.max(1)))
        last = int(np.argmax(us[:, 3]))
        print(f"   last exit: wave {last} (WG {last // 16}): stream done {us[last, 2]:.2f}, WG max done "
              f"{wg.max(1)[last // 16]:.2f}, exit {us[last, 3]:.2f}")
        # rank of wave within its WG (by finish) vs wave index in WG
        order = np.argsort(wg, axis=1)
        print("   mean finish by wave slot", " ".join(f"{x:5.1f}" for x in wg.mean(0)))
        xcd = np.arange(wg.shape[0]) % 8
        print("   WG max by blockIdx%8   ", " ".join(f"{wg.max(1)[xcd == k].mean():6.1f}" for k in range(8)))
        # dispatch order: entry and finish by blockIdx // 8 (position within its XCD), 8 bins
        pos = np.arange(wg.shape[0]) // 8
        bins = np.array_split(np.arange(pos.max() + 1), 8)
        print("   WG entry by dispatch pos", " ".join(f"{ent.min(1)[np.isin(pos, b)].mean():6.2f}" for b in bins))
        print("   WG done by dispatch pos ", " ".join(f"{wg.max(1)[np.isin(pos, b)].mean():6.2f}" for b in bins))
        print("   corr(entry, done) per WG  %.3f" % np.corrcoef(ent.min(1), wg.max(1))[0, 1])
        out_dir = os.path.join(ROOT, "gpurun_out")
        if os.path.isdir(out_dir):
            np.save(os.path.join(out_dir, f"stamps_{tag}_{it}.npy"), us)
            np.save(os.path.join(out_dir, f"stamps_{tag}_{it}_hw.npy"), raw[:, 4:6])


if __name__ == "__main__":
    main()
