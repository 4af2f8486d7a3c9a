"""GPU parity for the batched SHA-1 content hash (BASELINE config 5).

Oracle: hashlib.sha1 (OpenSSL) plus FIPS 180-4 known answers; the reference's
<sha1/sha1.h> (include/chunkio/cio_sha1.h:52) is third-party and not vendored,
so this path is pinned by the standard's vectors, not by reference fixtures.
"""
import hashlib

import numpy as np
import pytest

import chunkio_amd as cio
from chunkio_amd import workloads as wl

pytestmark = pytest.mark.gpu


def run(cuda, chunks, misalign=0):
    from test_gpu_crc import pack, to_dev
    buf, offs, lens = pack(chunks, misalign=[misalign] * len(chunks))
    return cio.sha1_batch_dev(to_dev(buf, cuda), offs, lens)


def test_fips_kats(cuda, golden):
    chunks = [bytes.fromhex(k["hex"]) for k in golden["sha1"]["kats"]]
    for mis in (0, 3):
        got = run(cuda, chunks, mis)
        assert [bytes(d).hex() for d in got] == [k["digest"] for k in golden["sha1"]["kats"]]


def test_padding_boundaries(cuda):
    rng = np.random.default_rng(21)
    lens = list(range(0, 200)) + [447, 448, 449, 511, 512, 513, 4095, 4096, 4097, 100003]
    chunks = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    for mis in (0, 1, 8):
        got = run(cuda, chunks, mis)
        for c, d in zip(chunks, got):
            assert bytes(d) == hashlib.sha1(c).digest(), len(c)


def test_cfg5_sample(cuda, golden, data400):
    import torch
    lens = wl.cfg2_lens(64)
    offs = wl.packed_offsets(lens)
    dev = torch.empty(wl.batch_bytes(offs, lens), dtype=torch.uint8, device=cuda)
    cio.fill_synthetic(dev, offs, lens, wl.CFG2_SEED)
    got = cio.sha1_batch_dev(dev, offs, lens)
    assert [bytes(d).hex() for d in got[:8]] == golden["sha1"]["cfg2_first8"]
    got400 = run(cuda, [data400])
    assert bytes(got400[0]).hex() == golden["sha1"]["400kb"]


def test_async_device_descriptors(cuda, golden):
    """cio_sha1_batch_dev_async (device-resident offsets/lengths, no sync) gives
    the digests of the synchronous entry on the full cfg5 batch, repeated on one
    stream, and on ragged lengths whose lanes end at different blocks."""
    import torch
    lens = wl.cfg2_lens()
    offs = wl.packed_offsets(lens, align=16)
    dev = torch.empty(wl.batch_bytes(offs, lens) + 64, dtype=torch.uint8, device=cuda)
    cio.fill_synthetic(dev, offs, lens, wl.CFG2_SEED)
    want = cio.sha1_batch_dev(dev, offs, lens)
    assert [bytes(d).hex() for d in want[:8]] == golden["sha1"]["cfg2_first8"]
    d_offs = torch.from_numpy(offs.astype(np.int64)).to(cuda)
    d_lens = torch.from_numpy(lens.astype(np.int64)).to(cuda)
    out = torch.zeros(len(lens) * 20, dtype=torch.uint8, device=cuda)
    for _ in range(3):
        cio.sha1_batch_dev_async(dev, d_offs, d_lens, out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().reshape(-1, 20), want)

    rng = np.random.default_rng(22)
    rl = rng.integers(0, 20000, 200).astype(np.uint64)
    ro = wl.packed_offsets(rl)
    rdev = torch.empty(wl.batch_bytes(ro, rl) + 64, dtype=torch.uint8, device=cuda)
    cio.fill_synthetic(rdev, ro, rl, 0x5A1)
    rout = torch.zeros(len(rl) * 20, dtype=torch.uint8, device=cuda)
    cio.sha1_batch_dev_async(rdev, torch.from_numpy(ro.astype(np.int64)).to(cuda),
                             torch.from_numpy(rl.astype(np.int64)).to(cuda), rout)
    got = rout.cpu().numpy().reshape(-1, 20)
    host = rdev.cpu().numpy()
    for i in range(len(rl)):
        assert bytes(got[i]) == hashlib.sha1(host[int(ro[i]):int(ro[i] + rl[i])].tobytes()).digest(), i


def test_many_workgroups_ragged_and_misaligned(cuda):
    """20,011 chunks (313 workgroups of 64 lanes, more than one per CU) with
    lengths 0..3000 at arbitrary byte offsets: lanes of one wave end at
    different blocks and most take the byte-wise message path."""
    import torch
    rng = np.random.default_rng(23)
    n = 20011
    lens = rng.integers(0, 3001, n).astype(np.uint64)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1] + rng.integers(0, 16, n - 1).astype(np.uint64))
    total = int(offs[-1] + lens[-1]) + 64
    host = rng.integers(0, 256, total, dtype=np.uint8)
    dev = torch.from_numpy(host).to(cuda)
    got = cio.sha1_batch_dev(dev, offs, lens)
    for i in range(n):
        o, ln = int(offs[i]), int(lens[i])
        assert bytes(got[i]) == hashlib.sha1(host[o:o + ln].tobytes()).digest(), i
