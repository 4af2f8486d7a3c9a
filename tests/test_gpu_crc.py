"""GPU parity: batched device CRC-32 (through the C ABI) vs the oracle / golden.

Bar: bit-exact raw CRC state for every chunk.  Sizes: the oracle runs on every
chunk up to config-2 size (1024 x 400 KB); at config-3/4 sizes the tests use
the golden samples plus size-independent properties (split-and-combine).
"""
import hashlib

import numpy as np
import pytest

import chunkio_amd as cio
from chunkio_amd import workloads as wl
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu
INIT = 0xFFFFFFFF


@pytest.fixture(autouse=True, params=["l64", "sub4"])
def layout(request, monkeypatch):
    """Every test in this module runs with both lane layouts of the CRC
    kernels: L64 (one 64-byte chain per lane, permlane transpose) and the
    4-sub-chain layout (CIO_GPU_L64 = 1 / 0, read at plan creation).  The
    library honours its A/B switches only under CIO_GPU_DIAG=1."""
    monkeypatch.setenv("CIO_GPU_DIAG", "1")
    monkeypatch.setenv("CIO_GPU_L64", "1" if request.param == "l64" else "0")
    return request.param


def to_dev(buf, cuda):
    import torch
    return torch.from_numpy(np.ascontiguousarray(buf)).to(cuda)


def pack(chunks, misalign=None, gap=0):
    """Place byte arrays in one buffer; chunk i starts at (16-aligned + misalign[i])."""
    offs, pos = [], 0
    for i, c in enumerate(chunks):
        m = 0 if misalign is None else int(misalign[i])
        pos = ((pos + 15) & ~15) + m
        offs.append(pos)
        pos += len(c) + gap
    buf = np.zeros(pos + 64, dtype=np.uint8)
    for o, c in zip(offs, chunks):
        buf[o:o + len(c)] = np.frombuffer(bytes(c), dtype=np.uint8) if not isinstance(c, np.ndarray) else c
    return buf, np.asarray(offs, np.uint64), np.asarray([len(c) for c in chunks], np.uint64)


def gpu_crc(cuda, buf, offs, lens, seeds=None):
    return cio.crc32_batch_dev(to_dev(buf, cuda), offs, lens, seeds=seeds)


def test_kats(cuda, golden, data400):
    from test_oracle import kat_bytes
    chunks = [kat_bytes(k, data400) for k in golden["kats"]]
    for mis in range(16):
        buf, offs, lens = pack(chunks, misalign=[mis] * len(chunks))
        got = gpu_crc(cuda, buf, offs, lens)
        assert [int(x) for x in got] == [k["raw"] for k in golden["kats"]], mis


def test_reference_fs_expectations(cuda, data400):
    # tests/fs.c:201-214: "\0\0" -> 0x41D912FF, "\0\0" + 400kb.txt -> 0x103CFA67
    buf, offs, lens = pack([b"\0\0", b"\0\0" + data400, b"\0\0" + data400 * 5], misalign=[6, 6, 6])
    got = gpu_crc(cuda, buf, offs, lens) ^ np.uint32(INIT)
    assert list(got) == [0x41D912FF, 0x103CFA67, 0x088740E7]


def test_every_length_0_to_4096(cuda, golden):
    g = golden["random_by_len"]
    chunks = [wl.gen_chunk(g["seed"], n, n) for n in range(g["max_len"] + 1)]
    for mis_mode in range(3):
        mis = [(n * 7 + mis_mode) % 16 for n in range(len(chunks))]
        buf, offs, lens = pack(chunks, misalign=mis)
        got = gpu_crc(cuda, buf, offs, lens)
        assert list(map(int, got)) == g["raw"]


def test_packed_contiguous_arbitrary_alignment(cuda):
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 20000, 3000).astype(np.uint64)
    buf, offs = wl.host_batch(0x77, lens)
    want = po.crc_batch(buf, offs, lens)
    got = gpu_crc(cuda, buf, offs, lens)
    np.testing.assert_array_equal(got, want)


def test_step_boundary_lengths_and_misalignments(cuda):
    lens = [4, 5, 6, 7, 8, 15, 16, 17, 63, 64, 65, 127, 128, 4031, 4032, 4033, 4095, 4096, 4097,
            4111, 8176, 8191, 8192, 8193, 12287, 12288, 12289, 65535, 65536, 65537, 262143, 409600]
    chunks, mis = [], []
    for m in range(16):
        for n in lens:
            chunks.append(wl.gen_chunk(0x99, len(chunks), n))
            mis.append(m)
    buf, offs, ln = pack(chunks, misalign=mis)
    want = po.crc_batch(buf, offs, ln)
    np.testing.assert_array_equal(gpu_crc(cuda, buf, offs, ln), want)


def test_seeds(cuda, golden):
    g = golden["seeded"]
    chunks = [wl.gen_chunk(g["data_seed"], v["len"], v["len"]) for v in g["vectors"]]
    seeds = np.asarray([v["seed"] for v in g["vectors"]], np.uint32)
    buf, offs, lens = pack(chunks, misalign=[i % 16 for i in range(len(chunks))])
    got = gpu_crc(cuda, buf, offs, lens, seeds=seeds)
    assert list(map(int, got)) == [v["raw"] for v in g["vectors"]]


def test_tiny_and_empty_chunks_with_seeds(cuda):
    rng = np.random.default_rng(6)
    chunks = [rng.integers(0, 256, n, dtype=np.uint8) for n in [0, 1, 2, 3, 0, 3, 4, 1] * 20]
    seeds = rng.integers(0, 2 ** 32, len(chunks), dtype=np.uint64).astype(np.uint32)
    buf, offs, lens = pack(chunks, misalign=rng.integers(0, 16, len(chunks)))
    want = po.crc_batch(buf, offs, lens, seeds=seeds)
    np.testing.assert_array_equal(gpu_crc(cuda, buf, offs, lens, seeds=seeds), want)
    # empty batch
    assert len(gpu_crc(cuda, np.zeros(16, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint64))) == 0


def test_zero_and_constant_data(cuda):
    # all-zero (the LDS tables' best case) and all-0xFF buffers, many sizes
    chunks = [np.zeros(n, np.uint8) for n in (4, 100, 4096, 70001)] + \
             [np.full(n, 0xFF, np.uint8) for n in (4, 100, 4096, 70001)]
    buf, offs, lens = pack(chunks, misalign=[3] * len(chunks))
    np.testing.assert_array_equal(gpu_crc(cuda, buf, offs, lens), po.crc_batch(buf, offs, lens))


def test_more_chunks_than_waves(cuda):
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 400, 20000).astype(np.uint64)
    buf, offs = wl.host_batch(0x1234, lens)
    np.testing.assert_array_equal(gpu_crc(cuda, buf, offs, lens), po.crc_batch(buf, offs, lens))


def test_overlapping_duplicate_and_unordered_chunks(cuda):
    """Descriptors are independent: chunks may overlap, repeat the same bytes,
    and come in any address order (a chunk's bytes are only read).  Both the
    stream kernel (long chunks) and the small kernel (<= 4 KiB), the device
    and the host batch."""
    rng = np.random.default_rng(31)
    buf = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
    for lo, hi in ((4, 4097), (4097, 600000)):
        lens = rng.integers(lo, hi, 300).astype(np.uint64)
        offs = rng.integers(0, len(buf) - hi - 16, 300).astype(np.uint64)
        offs[1::7] = offs[0::7][:len(offs[1::7])]            # duplicates of earlier descriptors
        lens[1::7] = lens[0::7][:len(lens[1::7])]
        offs[2::7] = offs[1::7][:len(offs[2::7])] + 3        # overlapping, shifted by 3 bytes
        order = np.argsort(-offs.astype(np.int64))            # descending addresses
        offs, lens = offs[order], lens[order]
        seeds = rng.integers(0, 2 ** 32, len(lens), dtype=np.uint64).astype(np.uint32)
        want = po.crc_batch(buf, offs, lens, seeds=seeds)
        np.testing.assert_array_equal(gpu_crc(cuda, buf, offs, lens, seeds=seeds), want, err_msg=f"dev {lo}")
        np.testing.assert_array_equal(cio.crc32_batch_host_packed(buf, offs, lens, seeds=seeds), want,
                                      err_msg=f"host {lo}")


def test_many_empty_chunks(cuda):
    """100,000 empty chunks: every CRC is its seed, no data is read."""
    n = 100000
    rng = np.random.default_rng(32)
    seeds = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    offs = rng.integers(0, 64, n).astype(np.uint64)
    lens = np.zeros(n, np.uint64)
    np.testing.assert_array_equal(gpu_crc(cuda, np.zeros(128, np.uint8), offs, lens, seeds=seeds), seeds)


def _uniform(n, ln, stride, mis, seed):
    """n chunks of ln bytes at mis + i * stride (a uniform batch)."""
    offs = (mis + np.arange(n, dtype=np.uint64) * np.uint64(stride)).astype(np.uint64)
    lens = np.full(n, ln, np.uint64)
    buf = np.zeros(int(offs[-1]) + ln + 64, np.uint8)
    rng = np.random.default_rng(seed)
    buf[:] = rng.integers(0, 256, buf.size, dtype=np.uint8)
    return buf, offs, lens


@pytest.mark.parametrize("ln,stride,mis", [
    (4096, 4096, 0),      # 4 KiB records: the register fold factor path
    (4090, 4096, 6),      # virtual length 4096 with a 6-byte head (chunk data at map+22 style offsets)
    (3000, 3008, 0),      # uniform partial step
    (4, 16, 0),           # smallest chunk that takes the stream path
    (4096, 4112, 5),      # virtual length 4101: two steps, main kernel
    (4081, 4096, 15),     # 15-byte head: head + seed reach granule 1 (register 1 of lane 0 in L64)
])
@pytest.mark.parametrize("l64", ["0", "1"])
def test_small_chunk_uniform_batches(cuda, monkeypatch, ln, stride, mis, l64):
    monkeypatch.setenv("CIO_GPU_L64", l64)
    buf, offs, lens = _uniform(9000, ln, stride, mis, seed=ln + mis)
    want = po.crc_batch(buf, offs, lens)
    np.testing.assert_array_equal(gpu_crc(cuda, buf, offs, lens), want)
    rng = np.random.default_rng(ln)
    seeds = rng.integers(0, 2 ** 32, len(lens), dtype=np.uint64).astype(np.uint32)
    np.testing.assert_array_equal(gpu_crc(cuda, buf, offs, lens, seeds=seeds),
                                  po.crc_batch(buf, offs, lens, seeds=seeds))


@pytest.mark.parametrize("l64", ["0", "1"])
def test_small_chunk_mixed_batch_and_kernel_agreement(cuda, monkeypatch, l64):
    # every chunk within one 4 KiB wave-step (virtual length <= 4096), with
    # tiny/empty chunks, random misalignment and seeds; the small-chunk kernel
    # and the stream kernel (CIO_GPU_SMALL=0) must agree with the oracle.
    monkeypatch.setenv("CIO_GPU_L64", l64)
    rng = np.random.default_rng(11)
    n = 30000
    mis = rng.integers(0, 16, n)
    lens = np.minimum(rng.integers(0, 4097, n), 4096 - mis)
    lens[::97] = 4096 - mis[::97]                                     # exactly one full step
    lens[::101] = rng.integers(0, 4, len(lens[::101]))                 # tiny / empty
    chunks = [wl.gen_chunk(0x5A11, i, int(m)) for i, m in enumerate(lens)]
    buf, offs, ln = pack(chunks, misalign=mis)
    seeds = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    want = po.crc_batch(buf, offs, ln, seeds=seeds)
    np.testing.assert_array_equal(gpu_crc(cuda, buf, offs, ln, seeds=seeds), want)
    monkeypatch.setenv("CIO_GPU_SMALL", "0")
    np.testing.assert_array_equal(gpu_crc(cuda, buf, offs, ln, seeds=seeds), want)


@pytest.mark.parametrize("l64", ["0", "1"])
def test_small_chunk_fewer_chunks_than_waves(cuda, monkeypatch, l64):
    monkeypatch.setenv("CIO_GPU_L64", l64)
    for n in (1, 2, 63, 4095, 4097):
        buf, offs, lens = _uniform(n, 4096, 4096, 0, seed=n)
        np.testing.assert_array_equal(gpu_crc(cuda, buf, offs, lens), po.crc_batch(buf, offs, lens))


@pytest.mark.parametrize("kind", ["cross_workgroup", "mixed_local", "fewer_steps_than_waves"])
def test_workgroup_local_and_cross_workgroup_pieces(cuda, kind):
    """Split chunks whose pieces all lie in one 16-wave workgroup are folded
    through LDS after the stream; the others take the global arrival.  These
    batches put both kinds side by side (and, for the last, empty wave ranges
    between a chunk's pieces), with seeds and head misalignment."""
    rng = np.random.default_rng(len(kind))
    if kind == "cross_workgroup":
        lens = np.full(64, 409600, np.uint64)            # ~64 waves per chunk
    elif kind == "mixed_local":
        lens = rng.integers(90_000, 120_000, 1100).astype(np.uint64)   # ~4 waves per chunk
    else:
        lens = rng.integers(1, 40_000, 40).astype(np.uint64)
    buf, offs = wl.host_batch(0x5EED + len(kind), lens)
    offs = offs + rng.integers(0, 16, len(offs)).astype(np.uint64)
    buf = np.concatenate([buf, np.zeros(32, np.uint8)])
    seeds = rng.integers(0, 2 ** 32, len(lens), dtype=np.uint64).astype(np.uint32)
    np.testing.assert_array_equal(gpu_crc(cuda, buf, offs, lens, seeds=seeds),
                                  po.crc_batch(buf, offs, lens, seeds=seeds))


@pytest.mark.parametrize("grid", [3, 4, 17])
def test_reduced_grid_split_paths(cuda, monkeypatch, grid):
    """Plans on fewer workgroups (CIO_GPU_GRID): 48 and 272 waves take the
    kernels' f64 even split, 64 the shift; uniform (stream and small kernel)
    and mixed batches, workgroup-local and cross-workgroup pieces, seeds."""
    monkeypatch.setenv("CIO_GPU_GRID", str(grid))
    rng = np.random.default_rng(grid)
    cases = [np.full(300, 409600, np.uint64),                      # uniform, stream kernel
             np.full(5000, 4096, np.uint64),                       # uniform, small kernel
             rng.integers(0, 300_000, 700).astype(np.uint64),      # mixed, tiny chunks too
             rng.integers(1, 4096, 3000).astype(np.uint64)]        # mixed, small kernel
    for k, lens in enumerate(cases):
        buf, offs = wl.host_batch(0x6A1D + k, lens, align=16)
        if k >= 2:
            offs = offs + rng.integers(0, 16, len(offs)).astype(np.uint64)
            buf = np.concatenate([buf, np.zeros(32, np.uint8)])
        seeds = rng.integers(0, 2 ** 32, len(lens), dtype=np.uint64).astype(np.uint32)
        np.testing.assert_array_equal(gpu_crc(cuda, buf, offs, lens, seeds=seeds),
                                      po.crc_batch(buf, offs, lens, seeds=seeds), err_msg=str(k))


@pytest.mark.parametrize("l64", ["0", "1"])
@pytest.mark.parametrize("grid", [None, 3])
def test_issue_ahead_uniform_aligned_batches(cuda, monkeypatch, grid, l64):
    """The issue-ahead stream kernel (uniform batches of whole 4 KiB steps at
    16-byte-aligned offsets: two ring slots, the refill issued once the
    current slot has landed, dummy refills past the range from chunk 0's
    first step) against the oracle and against the one-slot kernel
    (CIO_GPU_AHEAD=0): odd and even step counts per wave, one step per
    wave, fewer steps than waves, chunks spanning many waves and
    workgroups, seeds; on the full grid and a 48-wave grid (f64 split)."""
    if grid:
        monkeypatch.setenv("CIO_GPU_GRID", str(grid))
    monkeypatch.setenv("CIO_GPU_L64", l64)        # one 64-byte chain per lane (permlane transpose)
    rng = np.random.default_rng(91)
    cases = [(1, 4096 * 2), (5, 8192), (4097, 8192), (1000, 12288), (4096, 4096 * 3),
             (3, 4096 * 4099), (300, 409600), (2, 64 << 20)]
    for k, (n, ln) in enumerate(cases):
        lens = np.full(n, ln, np.uint64)
        buf, offs = wl.host_batch(0xA11E + k, lens, align=16)
        seeds = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32) if k % 2 else None
        want = po.crc_batch(buf, offs, lens, seeds=seeds)
        monkeypatch.setenv("CIO_GPU_AHEAD", "1")
        got = gpu_crc(cuda, buf, offs, lens, seeds=seeds)
        np.testing.assert_array_equal(got, want, err_msg=f"ahead {n}x{ln}")
        monkeypatch.setenv("CIO_GPU_AHEAD", "0")
        np.testing.assert_array_equal(gpu_crc(cuda, buf, offs, lens, seeds=seeds), want, err_msg=f"one-slot {n}x{ln}")


@pytest.mark.parametrize("grid", [None, "4x", 5])
def test_random_batches_property(cuda, monkeypatch, grid):
    """Randomised batches (fixed seeds, so a failure reproduces) through every
    plan path the geometry selects -- uniform aligned (issue-ahead), uniform
    misaligned, <= 4 KiB (small kernel), log-uniform mixed with empty and
    tiny chunks, one chunk over many waves -- with and without seeds, on the
    default grid, the 4-workgroups-per-CU grid and a 5-workgroup grid, in both
    lane layouts; every CRC against the oracle."""
    import torch
    if grid == "4x":
        monkeypatch.setenv("CIO_GPU_GRID", str(4 * torch.cuda.get_device_properties(cuda).multi_processor_count))
    elif grid is not None:
        monkeypatch.setenv("CIO_GPU_GRID", str(grid))
    rng = np.random.default_rng(0x5EED + (0 if grid is None else 7 if grid == "4x" else grid))
    cap = 48 << 20
    for k in range(12):
        kind = k % 5
        if kind == 0:                                   # uniform, whole 4 KiB steps, 16-aligned
            ln = 4096 * int(rng.integers(1, 200))
            lens = np.full(int(rng.integers(1, max(2, min(600, cap // ln)))), ln, np.uint64)
        elif kind == 1:                                 # uniform, any length
            ln = int(rng.integers(1, 300_000))
            lens = np.full(int(rng.integers(1, max(2, min(400, cap // ln)))), ln, np.uint64)
        elif kind == 2:                                 # small-chunk kernel
            lens = rng.integers(0, 4097, int(rng.integers(1, 20_000))).astype(np.uint64)
        elif kind == 3:                                 # log-uniform mixed, 0 B .. 8 MiB
            lens = np.floor(np.exp(rng.uniform(0, np.log(8 << 20), int(rng.integers(1, 300))))).astype(np.uint64)
            lens[rng.random(len(lens)) < 0.1] = 0
            lens = lens[np.cumsum(lens) <= cap] if lens.sum() > cap else lens
        else:                                           # one chunk over many waves, tiny ones around it
            lens = np.concatenate([rng.integers(0, 64, 5), [int(rng.integers(8 << 20, 40 << 20))],
                                   rng.integers(0, 64, 5)]).astype(np.uint64)
        if len(lens) == 0:
            lens = np.asarray([1], np.uint64)
        buf, offs = wl.host_batch(0xF00D + 31 * k, lens, align=16)
        if kind != 0:
            offs = offs + rng.integers(0, 16, len(offs)).astype(np.uint64)
            buf = np.concatenate([buf, np.zeros(32, np.uint8)])
        seeds = rng.integers(0, 2 ** 32, len(lens), dtype=np.uint64).astype(np.uint32) if k % 2 else None
        np.testing.assert_array_equal(gpu_crc(cuda, buf, offs, lens, seeds=seeds),
                                      po.crc_batch(buf, offs, lens, seeds=seeds),
                                      err_msg=f"batch {k} kind {kind} n {len(lens)} grid {grid}")


def test_one_huge_chunk_spans_all_waves(cuda):
    n = 48 * 1024 * 1024 + 12345
    data = wl.gen_chunk(0xBEEF, 0, n)
    buf, offs, lens = pack([data], misalign=[9])
    for seed in (INIT, 0, 0xDEADBEEF):
        got = gpu_crc(cuda, buf, offs, lens, seeds=np.asarray([seed], np.uint32))
        assert int(got[0]) == po.crc_update(seed, data)


def test_chunk_longer_than_4gib(cuda):
    """One chunk of 4 GiB + 4097 bytes (length and offsets past 32 bits),
    misaligned, between two small chunks, with and without a seed: zlib's
    CRC of the same bytes (the reference's crc_update takes a size_t length,
    crc32.c:337)."""
    import zlib
    import torch
    n = (4 << 30) + 4097
    lens = np.asarray([1000, n, 777], np.uint64)
    offs = np.asarray([3, 1024 + 5, 1024 + 5 + n + 11], np.uint64)
    dev = torch.empty(int(offs[-1] + lens[-1]) + 64, dtype=torch.uint8, device=cuda)
    cio.fill_synthetic(dev, offs, lens, 0x4C16)
    host = dev.cpu().numpy()
    want = [zlib.crc32(memoryview(host[int(o):int(o + ln)])) ^ INIT for o, ln in zip(offs, lens)]
    got = cio.crc32_batch_dev(dev, offs, lens)
    assert [int(x) for x in got] == want
    seeds = np.asarray([0x12345678, 0x9ABCDEF0, 0], np.uint32)
    got = cio.crc32_batch_dev(dev, offs, lens, seeds=seeds)
    want = [zlib.crc32(memoryview(host[int(o):int(o + ln)]), int(s) ^ INIT) ^ INIT
            for o, ln, s in zip(offs, lens, seeds)]
    assert [int(x) for x in got] == want


def test_plan_create_refuses_geometry_past_its_limits(cuda):
    """A chunk of more than 2^32 - 1 wave-steps (16 TiB) and a batch of 2^40
    wave-steps or more are refused at plan creation with a message; nothing is
    allocated for them (the lengths are never backed by memory)."""
    import ctypes
    lib = cio.lib()
    for lens, msg in (([1 << 45], b"chunk too large"), ([1 << 43] * 512, b"batch too large")):
        offs = (ctypes.c_uint64 * len(lens))(*([0] * len(lens)))
        ln = (ctypes.c_uint64 * len(lens))(*lens)
        h = ctypes.c_void_p()
        assert lib.cio_crc32_plan_create(ctypes.byref(h), offs, ln, len(lens)) == -1
        assert msg in lib.cio_gpu_last_error()
        assert not h.value


def test_plan_reuse_on_stream(cuda):
    import torch
    lens = wl.cfg2_lens(64)
    offs = wl.packed_offsets(lens)
    total = wl.batch_bytes(offs, lens)
    a = torch.empty(total, dtype=torch.uint8, device=cuda)
    b = torch.empty(total, dtype=torch.uint8, device=cuda)
    cio.fill_synthetic(a, offs, lens, wl.CFG2_SEED)
    cio.fill_synthetic(b, offs, lens, 0x5555)
    out = torch.empty(64, dtype=torch.int32, device=cuda)
    with cio.Crc32Plan(offs, lens) as plan:
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for buf, seed in ((a, wl.CFG2_SEED), (b, 0x5555), (a, wl.CFG2_SEED)):
                plan.exec(buf, out, stream=s)
                s.synchronize()
                got = out.cpu().numpy().view(np.uint32)
                want = po.crc_batch_chunks(seed, lens, idx=range(4))
                np.testing.assert_array_equal(got[:4], want)


def test_fill_matches_numpy_generator(cuda):
    import torch
    rng = np.random.default_rng(8)
    lens = rng.integers(0, 5000, 300).astype(np.uint64)
    buf, offs = wl.host_batch(0xF00D, lens)
    dev = torch.zeros(len(buf), dtype=torch.uint8, device=cuda)
    cio.fill_synthetic(dev, offs, lens, 0xF00D)
    np.testing.assert_array_equal(dev.cpu().numpy(), buf)


def test_cfg2_full_batch_golden(cuda, golden):
    import torch
    g = golden["cfg2"]
    lens = wl.cfg2_lens()
    offs = wl.packed_offsets(lens)
    dev = torch.empty(wl.batch_bytes(offs, lens), dtype=torch.uint8, device=cuda)
    cio.fill_synthetic(dev, offs, lens, g["seed"])
    got = cio.crc32_batch_dev(dev, offs, lens)
    assert list(map(int, got[:32])) == g["first32"]
    assert hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == g["sha256_of_raw_le"]


def split_combine_check(cuda, dev, offs, lens, want_full):
    """Size-independent property: CRC each chunk as two parts, fold on the host."""
    rng = np.random.default_rng(9)
    cut = (rng.random(len(lens)) * lens.astype(np.float64)).astype(np.uint64)
    offs2 = np.concatenate([offs, offs + cut])
    lens2 = np.concatenate([cut, lens - cut])
    seeds2 = np.concatenate([np.full(len(lens), INIT, np.uint32), np.zeros(len(lens), np.uint32)])
    parts = cio.crc32_batch_dev(dev, offs2, lens2, seeds=seeds2)
    n = len(lens)
    for i in range(0, n, max(1, n // 2000)):
        folded = cio.crc32_combine(int(parts[i]), int(parts[n + i]), int(lens2[n + i]))
        assert folded == int(want_full[i]), i


def test_cfg3_mixed_sizes_full(cuda, golden):
    import torch
    g = golden["cfg3"]
    lens = wl.cfg3_lens()
    offs = wl.packed_offsets(lens)          # contiguous: arbitrary chunk alignment
    dev = torch.empty(wl.batch_bytes(offs, lens) + 16, dtype=torch.uint8, device=cuda)
    cio.fill_synthetic(dev, offs, lens, g["seed"])
    got = cio.crc32_batch_dev(dev, offs, lens)
    assert [int(got[i]) for i in g["sample_idx"]] == g["sample_raw"]
    # every one of the 65,536 CRCs, against the reference crc32.c (make_golden.py)
    assert hashlib.sha256(got.astype("<u4").tobytes()).hexdigest() == g["sha256_of_raw_le"]
    split_combine_check(cuda, dev, offs, lens, got)


def test_plan_workgroups(cuda, monkeypatch):
    """Long batches (>= 4 MiB per wave: cfg3, cfg4 at one GPU) plan 4
    workgroups per CU, shorter ones (cfg2, 1024 x 4 MiB) one; CIO_GPU_GRID
    overrides.  (Parity of the 4x grid: test_cfg3_mixed_sizes_full and
    test_cfg4_full_job_sharded_g1_2_4_8's one-GPU shard take it.)"""
    cus = __import__("torch").cuda.get_device_properties(cuda).multi_processor_count
    l3 = wl.cfg3_lens()
    with cio.Crc32Plan(wl.packed_offsets(l3), l3) as p3:
        assert p3.workgroups == 4 * cus
    l2 = wl.cfg2_lens()
    with cio.Crc32Plan(wl.packed_offsets(l2, align=16), l2) as p2:
        assert p2.workgroups == cus
    l4 = np.full(1024, 4 << 20, np.uint64)      # uniform, 1 MiB per wave: one per CU
    with cio.Crc32Plan(wl.packed_offsets(l4), l4) as p4:
        assert p4.workgroups == cus
    l4 = np.full(8192, 4 << 20, np.uint64)      # cfg4 at one GPU, 8 MiB per wave: four
    with cio.Crc32Plan(wl.packed_offsets(l4), l4) as p4:
        assert p4.workgroups == 4 * cus
    monkeypatch.setenv("CIO_GPU_GRID", "17")
    with cio.Crc32Plan(wl.packed_offsets(l3), l3) as p3:
        assert p3.workgroups == 17


def test_stray_switches_without_the_gate_change_nothing(cuda, monkeypatch):
    """Without CIO_GPU_DIAG=1 the A/B switches are ignored: a deployment that
    carries CIO_GPU_GRID / _SMALL / _L64 / _AHEAD / _UNIFORM / _ANTICAMP /
    _PRIO by accident gets the shipped plans (same workgroups, same kernel)
    and the same CRCs.  With the gate the same switches do take effect."""
    import torch
    knobs = {"CIO_GPU_GRID": "17", "CIO_GPU_SMALL": "0", "CIO_GPU_L64": "0", "CIO_GPU_AHEAD": "0",
             "CIO_GPU_UNIFORM": "0", "CIO_GPU_ANTICAMP": "0", "CIO_GPU_PRIO": "0"}
    cases = {"cfg2": wl.cfg2_lens(), "cfg4k": np.full(4096, 4096, np.uint64),
             "camping": np.full(256 * 16 * 16, 4096, np.uint64)}
    monkeypatch.delenv("CIO_GPU_DIAG")
    for k in knobs:
        monkeypatch.delenv(k, raising=False)
    shipped = {}
    for name, lens in cases.items():
        offs = wl.packed_offsets(lens, align=16)
        with cio.Crc32Plan(offs, lens) as p:
            shipped[name] = (p.workgroups, p.kernel_name())
    dev = torch.empty(wl.batch_bytes(wl.packed_offsets(cases["cfg4k"], align=16), cases["cfg4k"]) + 64,
                      dtype=torch.uint8, device=cuda)
    offs = wl.packed_offsets(cases["cfg4k"], align=16)
    cio.fill_synthetic(dev, offs, cases["cfg4k"], 0x6A7E)
    want = po.crc_batch(dev.cpu().numpy(), offs, cases["cfg4k"])
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    for name, lens in cases.items():
        with cio.Crc32Plan(wl.packed_offsets(lens, align=16), lens) as p:
            assert (p.workgroups, p.kernel_name()) == shipped[name], (name, shipped[name])
    np.testing.assert_array_equal(cio.crc32_batch_dev(dev, offs, cases["cfg4k"]), want)
    monkeypatch.setenv("CIO_GPU_DIAG", "1")
    with cio.Crc32Plan(wl.packed_offsets(cases["cfg2"], align=16), cases["cfg2"]) as p:
        assert p.workgroups == 17
    with cio.Crc32Plan(offs, cases["cfg4k"]) as p:
        assert p.kernel_name() != shipped["cfg4k"][1]
    np.testing.assert_array_equal(cio.crc32_batch_dev(dev, offs, cases["cfg4k"]), want)


@pytest.mark.parametrize("clen,per_wave,reduced", [(4096, 16, True), (4096, 128, True), (4096, 25, False),
                                                   (4096, 256, False), (65536, 16, True), (65536, 64, True),
                                                   (65536, 25, False), (65536, 128, False)])
def test_anticamp_grid(cuda, monkeypatch, clen, per_wave, reduced):
    """Batches whose even split gives every wave the same multiple of 16 steps
    (small-chunk batches up to 128 chunks per wave, stream batches up to 64
    steps) plan one workgroup fewer per XCD (31 of every 32); the CRCs are the
    oracle's on both grids (CIO_GPU_ANTICAMP=0 keeps the full one)."""
    import torch
    cus = torch.cuda.get_device_properties(cuda).multi_processor_count
    if cus % 32:
        pytest.skip("grid not a multiple of 32 workgroups")
    steps = clen // 4096
    n = cus * 16 * per_wave // steps
    lens = np.full(n, clen, np.uint64)
    offs = wl.packed_offsets(lens, align=16)
    dev = torch.empty(wl.batch_bytes(offs, lens) + 64, dtype=torch.uint8, device=cuda)
    cio.fill_synthetic(dev, offs, lens, 0xCA4F + per_wave)
    host = dev.cpu().numpy()
    want = po.crc_batch(host, offs, lens) if n * clen <= (64 << 20) else None
    got = {}
    for env in ("1", "0"):
        monkeypatch.setenv("CIO_GPU_ANTICAMP", env)
        with cio.Crc32Plan(offs, lens) as p:
            assert p.workgroups == (cus // 32 * 31 if reduced and env == "1" else cus), env
            out = torch.empty(n, dtype=torch.int32, device=cuda)
            p.exec(dev, out)
            got[env] = out.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got["1"], got["0"])
    if want is not None:
        np.testing.assert_array_equal(got["1"], want)
    else:
        idx = np.arange(0, n, 997)
        np.testing.assert_array_equal(got["1"][idx], po.crc_batch(host, offs[idx], lens[idx]))


def test_read_stream_grids(cuda):
    """The read-only ceiling kernel (bench.py's roofline.read_stream) on one
    and four workgroups per CU and on a small grid; more than 4096
    workgroups is refused with a message, nothing launched."""
    import torch
    lib = cio.lib()
    buf = torch.zeros(64 << 20, dtype=torch.uint8, device=cuda)
    s = torch.cuda.current_stream(cuda).cuda_stream
    cus = torch.cuda.get_device_properties(cuda).multi_processor_count
    for wgs in (0, cus, 4 * cus, 3):
        assert lib.cio_gpu_read_stream_grid(buf.data_ptr(), buf.numel(), wgs, s) == 0
    assert lib.cio_gpu_read_stream(buf.data_ptr(), buf.numel(), s) == 0
    torch.cuda.synchronize(cuda)
    assert lib.cio_gpu_read_stream_grid(buf.data_ptr(), buf.numel(), 4097, s) != 0
    assert b"4096" in lib.cio_gpu_last_error()


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_ring_batches_overlap_same_results(cuda, depth):
    """cio_crc32_ring: batches queued on `depth` plans with their own streams,
    joined on the caller's stream, give every batch's CRCs (seeded and not),
    the same as one plan batch by batch; the batch queued after a caller-side
    write sees that write; depth outside 1..8 is refused."""
    import torch
    rng = np.random.default_rng(depth)
    lens = np.full(200, 409600, np.uint64)
    offs = wl.packed_offsets(lens, align=16)
    total = wl.batch_bytes(offs, lens)
    bufs = [torch.empty(total + 64, dtype=torch.uint8, device=cuda) for _ in range(5)]
    for b, t in enumerate(bufs):
        cio.fill_synthetic(t, offs, lens, 0x5EED + b)
    seeds_np = rng.integers(0, 2 ** 32, len(lens), dtype=np.uint64).astype(np.uint32)
    seeds = torch.from_numpy(seeds_np.view(np.int32)).to(cuda)
    outs = [torch.empty(len(lens), dtype=torch.int32, device=cuda) for _ in range(10)]
    with cio.Crc32Ring(offs, lens, depth=depth) as ring:
        for k in range(10):
            if k == 7:
                bufs[k % 5][int(offs[3]) + 5] ^= 0xFF      # a caller-side write the next batch must see
            ring.exec(bufs[k % 5], outs[k], seeds=seeds if k % 2 else None)
        ring.join()
    torch.cuda.synchronize(cuda)
    with cio.Crc32Plan(offs, lens) as plan:
        for k in range(10):
            want = torch.empty_like(outs[k])
            plan.exec(bufs[k % 5], want, seeds=seeds if k % 2 else None)
            torch.cuda.synchronize(cuda)
            if k < 7 and k % 5 == 2:
                continue    # batch 2's buffer was changed after it ran
            assert torch.equal(outs[k], want), k
    host = bufs[2].cpu().numpy()
    assert int(outs[7].cpu().numpy().view(np.uint32)[3]) == po.crc_batch(host, offs[3:4], lens[3:4],
                                                                          seeds=seeds_np[3:4])[0]
    for bad in (0, 9):
        with pytest.raises(cio.CioGpuError):
            cio.Crc32Ring(offs, lens, depth=bad)


def test_ring_runs_on_its_own_device_and_restores_the_callers(cuda):
    """A ring belongs to the device current at create: exec / join / close
    after the caller switched devices (cio_gpu_set_device to another ordinal,
    ordinal 0 again on a one-GPU box) still run on the ring's device, give
    the plan's CRCs, and leave the caller's device current."""
    import torch
    lib = cio.lib()
    ndev = cio.device_count()
    lens = np.full(64, 409600, np.uint64)
    offs = wl.packed_offsets(lens, align=16)
    buf = torch.empty(wl.batch_bytes(offs, lens) + 64, dtype=torch.uint8, device=cuda)
    cio.fill_synthetic(buf, offs, lens, 0x77)
    want = po.crc_batch(buf.cpu().numpy(), offs, lens)
    out = torch.empty(len(lens), dtype=torch.int32, device=cuda)
    assert lib.cio_gpu_set_device(0) == 0
    ring = cio.Crc32Ring(offs, lens, depth=2)
    other = 1 % ndev
    try:
        assert lib.cio_gpu_set_device(other) == 0
        s = torch.cuda.current_stream(cuda)
        ring.exec(buf, out, stream=s)
        assert lib.cio_gpu_get_device() == other
        ring.join(stream=s)
        assert lib.cio_gpu_get_device() == other
        torch.cuda.synchronize(cuda)
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)
    finally:
        ring.close()
        assert lib.cio_gpu_get_device() == other
        lib.cio_gpu_set_device(0)


@pytest.mark.parametrize("ndev", [1, 2, 3, 8])
def test_split_one_buffer_over_devices(cuda, ndev):
    """cio_crc32_split_host_multi: one buffer cut into a piece per (logical)
    device, the piece states joined with cio_crc32_combine, equals crc_update
    over the whole buffer, seeded or not; lengths below one piece per device,
    not a 4 KiB multiple, and empty."""
    rng = np.random.default_rng(ndev)
    for ln in (0, 1, 4095, 4096 * ndev + 7, 3 << 20, (64 << 20) + 12345):
        buf = rng.integers(0, 256, ln, dtype=np.uint8)
        for seed in (cio.CRC_INIT, 0x1234ABCD):
            want = po.crc_batch(buf, np.zeros(1, np.uint64), np.full(1, ln, np.uint64),
                                seeds=np.full(1, seed, np.uint32))[0]
            assert cio.crc32_split_host(buf, seed, devices=[0] * ndev) == want, (ln, seed)


def test_cfg4_shard_golden(cuda, golden):
    import torch
    g = golden["cfg4"]
    idx = np.arange(64)                       # first 64 chunks (one GPU of a G=128 split)
    lens = wl.cfg4_lens()[idx]
    offs = wl.packed_offsets(lens)
    dev = torch.empty(wl.batch_bytes(offs, lens), dtype=torch.uint8, device=cuda)
    cio.fill_synthetic(dev, offs, lens, g["seed"])
    got = cio.crc32_batch_dev(dev, offs, lens)
    assert list(map(int, got[:8])) == g["sample_raw"]
    split_combine_check(cuda, dev, offs, lens, got)


def test_cfg4_full_job_sharded_g1_2_4_8(cuda, golden):
    """BASELINE config 4 at full size (8192 x 4 MiB = 34.4 GB) as the G = 1, 2, 4
    and 8 GPU jobs see it: shard r holds chunks r, r+G, ... (shard.shard_ids), is
    filled by generator chunk id into its own packed buffer, and is CRC'd as one
    batch; shard.assemble scatters the results back to chunk order, and the
    digest of all 8192 CRCs must equal the one made from the reference crc32.c
    (tests/golden/make_golden.py).  One GPU runs the shards one after another."""
    import torch
    from chunkio_amd import shard
    g = golden["cfg4"]
    n, ln = g["n"], g["len"]
    dev = torch.empty(n * ln, dtype=torch.uint8, device=cuda)
    for world in (1, 2, 4, 8):
        parts = []
        for r in range(world):
            ids = shard.shard_ids(n, r, world)
            lens = np.full(len(ids), ln, np.uint64)
            offs = np.arange(len(ids), dtype=np.uint64) * np.uint64(ln)
            cio.fill_synthetic(dev, offs, lens, g["seed"], ids=ids)
            parts.append(cio.crc32_batch_dev(dev, offs, lens))
        full = shard.assemble(n, world, parts)
        assert list(map(int, full[:8])) == g["sample_raw"], world
        assert hashlib.sha256(full.astype("<u4").tobytes()).hexdigest() == g["sha256_of_raw_le"], world
    del dev
    torch.cuda.empty_cache()


@pytest.mark.parametrize("cfg", ["cfg2", "cfg4k", "cfg3", "sha1"])
def test_weak_jobs_sharded_g2_8(cuda, golden, cfg):
    """The weak-scaled jobs bench.py --gpus N runs (N x the per-GPU batch,
    chunk i on rank i mod N) at N = 2 and 8, every rank's shard built exactly
    as bench.geometry builds it and run one after another on this GPU; the
    gathered job must equal the reference digest of that job
    (tests/golden/make_golden.py weak_jobs: crc32.c + zlib, hashlib for SHA-1).
    cfg3 at N = 8 is 318 GB of chunks, 40 GB at a time."""
    import torch
    import bench
    from chunkio_amd import shard
    from chunkio_amd import workloads as wl
    dev = None
    for world in (2, 8):
        parts = []
        for r in range(world):
            lens, ids, seed, _, scaling = bench.geometry(cfg, r, world)
            assert scaling == "weak"
            offs = wl.packed_offsets(lens, align=16)
            need = wl.batch_bytes(offs, lens) + 64
            if dev is None or dev.numel() < need:
                dev = None
                torch.cuda.empty_cache()
                dev = torch.empty(need, dtype=torch.uint8, device=cuda)
            cio.fill_synthetic(dev, offs, lens, seed, ids=ids)
            if cfg == "sha1":
                parts.append(cio.sha1_batch_dev(dev, offs, lens).reshape(-1, 20))
            else:
                parts.append(cio.crc32_batch_dev(dev, offs, lens))
        n = sum(len(p) for p in parts)
        if cfg == "sha1":
            job = np.empty((n, 20), np.uint8)
            for r, p in enumerate(parts):
                job[shard.shard_ids(n, r, world)] = p
            got = hashlib.sha256(job.tobytes()).hexdigest()
        else:
            got = hashlib.sha256(shard.assemble(n, world, parts).astype("<u4").tobytes()).hexdigest()
        assert got == golden["weak_jobs"][cfg][str(world)], (cfg, world)
    del dev
    torch.cuda.empty_cache()


def test_host_batch_end_to_end(cuda, data400):
    rng = np.random.default_rng(10)
    bufs = [np.frombuffer(b"\0\0" + data400, np.uint8)]
    bufs += [rng.integers(0, 256, int(n), dtype=np.uint8) for n in rng.integers(0, 300000, 200)]
    big = rng.integers(0, 256, 150 * 1024 * 1024 + 7, dtype=np.uint8)   # spans 3 staging groups
    bufs += [big[1:]]                                                   # misaligned host view
    bufs += [np.zeros(0, np.uint8), np.frombuffer(b"abc", np.uint8)]
    seeds = rng.integers(0, 2 ** 32, len(bufs), dtype=np.uint64).astype(np.uint32)
    got = cio.crc32_batch_host(bufs, seeds=seeds)
    want = [po.crc_update(int(s), b) for s, b in zip(seeds, bufs)]
    assert list(map(int, got)) == want
    got0 = cio.crc32_batch_host(bufs[:1])
    assert int(got0[0]) ^ INIT == 0x103CFA67


def test_host_batch_packed_and_graduated_groups(cuda):
    # One packed host array through crc32_batch_host_packed (pointer array
    # built in numpy); sizes straddle the graduated first groups (4, 8, 16 ...
    # MiB) and one chunk spans several of them.
    rng = np.random.default_rng(13)
    lens = rng.integers(0, 3_000_000, 120).astype(np.uint64)
    lens[7] = 40 * 1024 * 1024 + 3
    lens[::17] = rng.integers(0, 4, len(lens[::17]))
    host, offs = wl.host_batch(0x9AC, lens, align=1)
    seeds = rng.integers(0, 2 ** 32, len(lens), dtype=np.uint64).astype(np.uint32)
    want = po.crc_batch(host, offs, lens, seeds=seeds)
    np.testing.assert_array_equal(cio.crc32_batch_host_packed(host, offs, lens, seeds=seeds), want)
    np.testing.assert_array_equal(cio.crc32_batch_host_packed(host, offs, lens, seeds=seeds, devices=[0, 0]), want)
    bufs = [host[int(o):int(o) + int(n)] for o, n in zip(offs, lens)]
    np.testing.assert_array_equal(cio.crc32_batch_host(bufs, seeds=seeds), want)


@pytest.mark.gpu
def test_host_plan_cache_same_geometry_new_data(cuda):
    """The host pipeline caches plan images by geometry (host_pipeline.hip
    PlanImage): repeated calls of one geometry with different bytes and seeds,
    interleaved with a geometry that differs in one length and one that
    differs only in chunk order (a permutation: same offsets set, other
    ids), must each give the oracle's CRCs."""
    rng = np.random.default_rng(31)
    lens = rng.integers(1, 2_000_000, 150).astype(np.uint64)
    offs = wl.packed_offsets(lens, align=16)
    total = wl.batch_bytes(offs, lens) + 16
    lens2 = lens.copy()
    lens2[77] -= 1
    perm = rng.permutation(len(lens))
    for rep in range(3):
        host = rng.integers(0, 256, total, dtype=np.uint8)
        seeds = rng.integers(0, 2 ** 32, len(lens), dtype=np.uint64).astype(np.uint32)
        for o, ln in ((offs, lens), (offs, lens2), (offs[perm], lens[perm])):
            want = po.crc_batch(host, o, ln, seeds=seeds)
            np.testing.assert_array_equal(cio.crc32_batch_host_packed(host, o, ln, seeds=seeds), want)


@pytest.mark.gpu
def test_host_plan_cache_admission_and_byte_cap(cuda):
    """The plan image cache stores a geometry on its second sighting only and
    stays under its byte cap: 40 host batches that never repeat a geometry
    store nothing and leave the held bytes where they were; one geometry
    called three times is stored once and hit once; 60 distinct geometries
    each seen twice keep every pipeline under CIO_GPU_PLAN_CACHE_MB (16)."""
    rng = np.random.default_rng(77)
    s0 = cio.plan_cache_stats()
    for k in range(40):
        lens = rng.integers(1, 300_000, 64 + k).astype(np.uint64)
        host, offs = wl.host_batch(0x51 + k, lens, align=16)
        want = po.crc_batch(host, offs, lens)
        np.testing.assert_array_equal(cio.crc32_batch_host_packed(host, offs, lens), want)
    s1 = cio.plan_cache_stats()
    assert s1["stores"] == s0["stores"] and s1["bytes"] == s0["bytes"], (s0, s1)
    assert s1["misses"] - s0["misses"] >= 40
    lens = rng.integers(1, 300_000, 50).astype(np.uint64)
    host, offs = wl.host_batch(0x99, lens, align=16)
    want = po.crc_batch(host, offs, lens)
    for _ in range(3):
        np.testing.assert_array_equal(cio.crc32_batch_host_packed(host, offs, lens), want)
    groups = cio.pipe_last_timing()["groups"]     # staging groups per call: one geometry each
    s2 = cio.plan_cache_stats()
    assert s2["stores"] - s1["stores"] == groups and s2["hits"] - s1["hits"] >= groups, (groups, s1, s2)
    # small chunks make large images (~1.3 MB per 64 MiB group of 4 KiB chunks)
    for k in range(60):
        lens = np.full(2000 + 37 * k, 4096 - (k % 7), dtype=np.uint64)
        host, offs = wl.host_batch(0x700 + k, lens, align=16)
        for _ in range(2):
            cio.crc32_batch_host_packed(host, offs, lens)
    s3 = cio.plan_cache_stats()
    assert s3["stores"] > s2["stores"] and s3["evictions"] > s2["evictions"], (s2, s3)
    assert s3["bytes"] <= 16 * (1 << 20) * s3["pipelines"], s3
    assert s3["entries"] <= 32 * s3["pipelines"], s3


def test_host_pipeline_reuse_and_growth(cuda):
    """The persistent host pipeline across calls whose shapes grow and shrink
    (plan arenas reallocated, counters re-zeroed, state array regrown)."""
    rng = np.random.default_rng(11)
    for count, hi in ((3, 5000), (20000, 4100), (7, 9_000_000), (1, 64), (5000, 20000)):
        bufs = [rng.integers(0, 256, int(n), dtype=np.uint8) for n in rng.integers(0, hi, count)]
        got = cio.crc32_batch_host(bufs)
        want = [po.crc_update(INIT, b) for b in bufs]
        assert list(map(int, got)) == want, (count, hi)


@pytest.mark.gpu
def test_host_pipeline_concurrent_callers(cuda):
    """Four host threads on one device: each takes its own pooled pipeline."""
    import threading
    rng = np.random.default_rng(12)
    jobs = [[rng.integers(0, 256, int(n), dtype=np.uint8) for n in rng.integers(1, 400000, 300)]
            for _ in range(4)]
    results = [None] * len(jobs)

    def run(k):
        results[k] = cio.crc32_batch_host(jobs[k])

    th = [threading.Thread(target=run, args=(k,)) for k in range(len(jobs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for k, bufs in enumerate(jobs):
        assert list(map(int, results[k])) == [po.crc_update(INIT, b) for b in bufs]


def test_device_batches_from_concurrent_threads(cuda):
    """Eight threads each run device batches (their own plans and streams, the
    small and the stream kernel) at the same time as the others."""
    import threading
    import torch
    rng = np.random.default_rng(13)
    jobs = []
    for k in range(8):
        lens = rng.integers(0, 4097 if k % 2 else 300000, 400).astype(np.uint64)
        buf, offs = wl.host_batch(0x7000 + k, lens)
        jobs.append((buf, offs, lens, po.crc_batch(buf, offs, lens)))
    errors = []

    def run(k):
        try:
            buf, offs, lens, want = jobs[k]
            dev = torch.from_numpy(buf).to(cuda)
            torch.cuda.synchronize(cuda)      # the upload (current stream) before the batches on s
            s = torch.cuda.Stream(device=cuda)
            for _ in range(5):
                got = cio.crc32_batch_dev(dev, offs, lens, stream=s)
                if not np.array_equal(got, want):
                    errors.append(k)
        except Exception as e:     # reported below
            errors.append((k, repr(e)))

    th = [threading.Thread(target=run, args=(k,)) for k in range(len(jobs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors


@pytest.mark.gpu
def test_host_registered_ranges_direct_dma(cuda, tmp_path):
    """Chunks inside ranges pinned in place (cio_crc32_host_register) are
    DMA'd directly; groups mixing registered and unregistered chunks are
    staged.  Results are identical either way.  Covers an anonymous buffer and
    a MAP_SHARED file mapping (chunkio's own buffers, cio_file_unix.c:100)."""
    import mmap
    rng = np.random.default_rng(13)
    anon = mmap.mmap(-1, 96 << 20)
    a = np.frombuffer(anon, dtype=np.uint8)
    a[:] = rng.integers(0, 256, a.size, dtype=np.uint8)
    path = tmp_path / "chunks.bin"
    path.write_bytes(rng.integers(0, 256, 8 << 20, dtype=np.uint8).tobytes())
    fd = open(path, "r+b")
    fmap = mmap.mmap(fd.fileno(), 0, mmap.MAP_SHARED)
    f = np.frombuffer(fmap, dtype=np.uint8)
    loose = rng.integers(0, 256, 300000, dtype=np.uint8)
    cuts = np.sort(rng.integers(0, a.size, 60))
    bufs = [a[int(x):int(y)] for x, y in zip(cuts[:-1], cuts[1:])]       # adjacent runs
    bufs += [a[5:409605], f[3:4000003], f[4000003:], a[:0], loose]
    want = [po.crc_update(INIT, b) for b in bufs]
    before = cio.crc32_batch_host(bufs)
    cio.host_register(a)
    try:
        file_ok = True
        try:
            cio.host_register(f)
        except cio.CioGpuError:
            file_ok = False            # the driver may refuse file-backed pages
        with pytest.raises(cio.CioGpuError):
            cio.host_register(a)       # already registered
        got = cio.crc32_batch_host(bufs)
        only_a = cio.crc32_batch_host(bufs[:59])                         # all-registered groups
        if file_ok:
            cio.host_unregister(f)
    finally:
        cio.host_unregister(a)
    with pytest.raises(cio.CioGpuError):
        cio.host_unregister(a)
    assert list(map(int, before)) == want
    assert list(map(int, got)) == want
    assert list(map(int, only_a)) == want[:59]
    fd.close()


@pytest.mark.gpu
def test_cfg2_tiled_400kb_full_size(cuda, data400):
    """SURVEY §8(d) sanity batch at the full cfg2 size: 400kb.txt tiled
    1024 times, every CRC finalizes to 0x777A8F30 (known answer, §8(c))."""
    d = np.frombuffer(data400, np.uint8)
    n = 1024
    offs = np.arange(n, dtype=np.uint64) * np.uint64(d.size)
    lens = np.full(n, d.size, dtype=np.uint64)
    got = gpu_crc(cuda, np.tile(d, n), offs, lens)
    assert np.all((got ^ np.uint32(0xFFFFFFFF)) == np.uint32(0x777A8F30))


@pytest.mark.gpu
def test_host_batch_multi_device_logical(cuda):
    """cio_crc32_batch_host_multi with G logical devices mapped onto the
    box's GPU(s): chunk i -> devices[i % G], one host thread + pipeline per
    entry, results scattered back by index; equal to the oracle and to the
    single-device call for G = 1, 2, 3, 5 (more entries than chunks too)."""
    rng = np.random.default_rng(21)
    bufs = [rng.integers(0, 256, int(n), dtype=np.uint8) for n in rng.integers(0, 600000, 257)]
    bufs += [np.zeros(0, np.uint8), rng.integers(0, 256, 70 << 20, dtype=np.uint8)]   # spans groups
    seeds = rng.integers(0, 2 ** 32, len(bufs), dtype=np.uint64).astype(np.uint32)
    want = [po.crc_update(int(s), b) for s, b in zip(seeds, bufs)]
    ndev = max(1, cio.device_count())
    for g in (1, 2, 3, 5):
        devs = [k % ndev for k in range(g)]
        got = cio.crc32_batch_host(bufs, seeds=seeds, devices=devs)
        assert list(map(int, got)) == want, g
    few = cio.crc32_batch_host(bufs[:2], devices=[0] * 4)
    assert list(map(int, few)) == [po.crc_update(INIT, b) for b in bufs[:2]]
    with pytest.raises(cio.CioGpuError):
        cio.crc32_batch_host(bufs[:2], devices=[ndev + 7])


@pytest.mark.gpu
def test_plan_survives_other_device_init(cuda):
    """the per-device tables a plan points to must not move
    when another device is first used.  Create a plan on device 0, initialise
    every other visible device, then re-execute the plan."""
    import ctypes
    import torch
    rng = np.random.default_rng(22)
    lens = rng.integers(0, 300000, 64).astype(np.uint64)
    host, offs = wl.host_batch(7, lens, align=16)
    base = torch.from_numpy(host).to(cuda)
    plan = cio.Crc32Plan(offs, lens)
    out = torch.empty(len(lens), dtype=torch.int32, device=cuda)
    plan.exec(base, out)
    torch.cuda.synchronize()
    first = out.cpu().numpy().view(np.uint32).copy()
    lib = cio.lib()
    for d in range(1, cio.device_count()):
        assert lib.cio_gpu_set_device(d) == 0 and lib.cio_gpu_init() == 0
    assert lib.cio_gpu_set_device(0) == 0
    plan.exec(base, out)
    torch.cuda.synchronize()
    again = out.cpu().numpy().view(np.uint32)
    assert np.array_equal(first, again)
    assert list(map(int, first)) == [po.crc_update(INIT, host[int(o):int(o + n)]) for o, n in zip(offs, lens)]
    plan.close()
    del ctypes


@pytest.mark.gpu
def test_verify_paths_multi_device_and_delete(cuda, tmp_path, data400):
    """cio_verify_paths_multi over logical devices: same verdicts as one
    device; CIO_DELETE_IRRECOVERABLE removes exactly the corrupted files."""
    from chunkio_amd import chunkfile as cf
    paths = []
    for i in range(40):
        p = str(tmp_path / "s" / f"c{i:02d}")
        c, _ = cf.ChunkFile.open(p, deferred_crc=True)
        c.write(data400[: 10000 * (i + 1)])
        c.close()
        paths.append(p)
    bad = {3: 24 + 77, 17: 3, 31: 0}          # content byte, CRC byte, magic
    for i, off in bad.items():
        raw = bytearray(open(paths[i], "rb").read())
        raw[off] ^= 0x11
        open(paths[i], "wb").write(bytes(raw))
    st1, er1, cr1 = cf.verify_paths(paths)
    ndev = max(1, cio.device_count())
    st2, er2, cr2 = cf.verify_paths(paths, devices=[k % ndev for k in range(3)])
    assert np.array_equal(st1, st2) and np.array_equal(er1, er2) and np.array_equal(cr1, cr2)
    assert [i for i in range(40) if st1[i] != cf.CIO_OK] == sorted(bad)
    assert [int(er1[i]) for i in sorted(bad)] == [cf.CIO_ERR_BAD_CHECKSUM, cf.CIO_ERR_BAD_CHECKSUM,
                                                 cf.CIO_ERR_BAD_LAYOUT]
    st3, _, _ = cf.verify_paths(paths, flags=cf.CIO_CHECKSUM | cf.CIOA_VERIFY_DELETE_IRRECOVERABLE,
                                devices=[0, 0])
    assert np.array_equal(st3, st1)
    import os
    assert [i for i in range(40) if not os.path.exists(paths[i])] == sorted(bad)


@pytest.mark.gpu
def test_verify_paths_large_files_across_staging_groups(cuda, tmp_path):
    """Chunk files written here byte by byte (header per cio_file.c:45-60 /
    cio_file_st.h, CRC from zlib over [22, 24 + meta + content)), not by this
    library: a 150 MB chunk whose CRC region spans several staging groups of
    the file-range pipeline (4, 8, 16, 32, 64 MiB), a 70 MB one with
    metadata, small ones between them, and one flipped byte deep inside the
    large file.  cio_verify_paths must pass exactly the intact files and
    return their raw CRC states."""
    import struct
    import zlib
    from chunkio_amd import chunkfile as cf
    rng = np.random.default_rng(31)

    def chunk_file(path, content, meta=b""):
        region = struct.pack(">H", len(meta)) + meta + content
        crc = zlib.crc32(region)
        hdr = bytes([0xC1, 0x00]) + struct.pack(">I", crc) + bytes(4) + struct.pack(">I", len(content)) + bytes(8)
        with open(path, "wb") as f:
            f.write(hdr + region)
        return crc

    sizes = [150_000_003, 4096, 70_000_000, 1, 3_000_000, 0]
    metas = [b"", b"m", b"meta-" * 300, b"", b"xy", b""]
    paths, crcs = [], []
    for i, (n, m) in enumerate(zip(sizes, metas)):
        p = str(tmp_path / f"chunk{i}")
        crcs.append(chunk_file(p, rng.integers(0, 256, n, dtype=np.uint8).tobytes(), m))
        paths.append(p)
    st, er, raw = cf.verify_paths(paths)
    assert list(st) == [cf.CIO_OK] * len(paths), (list(st), list(er))
    assert [int(r) ^ 0xFFFFFFFF for r in raw] == crcs
    # one flipped byte 100 MB into the big file's content: only it fails
    with open(paths[0], "r+b") as f:
        f.seek(24 + 100_000_000)
        b = f.read(1)
        f.seek(24 + 100_000_000)
        f.write(bytes([b[0] ^ 0x40]))
    st, er, raw = cf.verify_paths(paths)
    assert int(st[0]) == cf.CIO_CORRUPTED and int(er[0]) == cf.CIO_ERR_BAD_CHECKSUM
    assert list(st[1:]) == [cf.CIO_OK] * (len(paths) - 1)
    assert [int(r) ^ 0xFFFFFFFF for r in raw[1:]] == crcs[1:]


def test_pci_bus_id_names_the_device(cuda):
    """cio_gpu_pci_bus_id: the PCI address of an ordinal, as the bench's
    topology records it ("dddd:bb:dd.f"); agrees with torch's device
    properties; a short buffer is refused with a message."""
    import ctypes
    import re
    import torch
    lib = cio.lib()
    buf = ctypes.create_string_buffer(64)
    assert lib.cio_gpu_pci_bus_id(0, buf, 64) == 0
    bus = buf.value.decode()
    assert re.fullmatch(r"[0-9a-f]{4}:[0-9a-f]{2}:[0-9a-f]{2}\.[0-9a-f]", bus.lower()), bus
    p = torch.cuda.get_device_properties(0)
    if hasattr(p, "pci_bus_id"):
        assert int(bus.split(":")[1], 16) == int(p.pci_bus_id), (bus, p.pci_bus_id)
    assert lib.cio_gpu_pci_bus_id(0, buf, 8) != 0
    assert b"13 bytes" in lib.cio_gpu_last_error()
