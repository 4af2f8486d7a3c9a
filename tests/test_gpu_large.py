"""GPU parity at the largest sizes: chunks longer than 2^32 bytes and chunks
that start past 4 GiB in the batch buffer.

Everything the plan and the kernels carry per chunk is 64-bit (offsets,
lengths, step numbers, the x^(8 n) exponents that shift partial CRCs); the
BASELINE batches reach 39.7 GB (cfg3) but no single chunk there passes 4 MiB.
Here one chunk is 4 GiB + 4099 bytes at a misaligned start, followed by small
chunks whose offsets are above 2^32.  The oracle is the C restatement
(oracle/crc32_oracle.c via oracle.pyoracle) over the same bytes copied back
to the host.
"""
import numpy as np
import pytest

import chunkio_amd as cio
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu
INIT = 0xFFFFFFFF


def _batch():
    big = (1 << 32) + 4099
    lens = np.array([big, 5000, 3, 0, 409600, 17], np.uint64)
    offs = np.zeros(len(lens), np.uint64)
    pos = 5                                      # misaligned first chunk
    for i, ln in enumerate(lens):
        offs[i] = pos
        pos += int(ln) + 7 + i                   # ragged gaps: every later offset misaligned
    return offs, lens, pos + 64


def test_chunk_longer_than_4gib_and_offsets_past_4gib(cuda, monkeypatch):
    import torch
    offs, lens, total = _batch()
    gen = torch.Generator(device=cuda)
    gen.manual_seed(0x4B16)
    dev = torch.randint(0, 256, (total,), dtype=torch.uint8, device=cuda, generator=gen)
    host = dev.cpu().numpy()
    seeds = np.array([INIT, 0, 0xDEADBEEF, INIT, 0x12345678, INIT], np.uint32)
    want = np.array([po.crc_update(int(s), host[int(o):int(o + n)]) for s, o, n in zip(seeds, offs, lens)],
                    np.uint32)
    # both lane layouts of the stream kernel
    monkeypatch.setenv("CIO_GPU_DIAG", "1")
    for l64 in ("1", "0"):
        monkeypatch.setenv("CIO_GPU_L64", l64)
        got = cio.crc32_batch_dev(dev, offs, lens, seeds=seeds)
        np.testing.assert_array_equal(got, want, err_msg=f"device batch, CIO_GPU_L64={l64}")
    del dev
    torch.cuda.empty_cache()
    # the host pipeline: the big chunk crosses ~65 staging groups, its state chained between them
    got_h = cio.crc32_batch_host_packed(host, offs, lens, seeds=seeds)
    np.testing.assert_array_equal(got_h, want, err_msg="host batch")
    # crc32_combine with a tail longer than 2^32 bytes
    a = po.crc_update(INIT, host[5:5 + 1000])
    b0 = po.crc_update(0, host[5 + 1000:5 + int(lens[0])])
    assert cio.crc32_combine(a, b0, int(lens[0]) - 1000) == int(want[0])
