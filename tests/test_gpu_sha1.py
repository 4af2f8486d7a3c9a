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
