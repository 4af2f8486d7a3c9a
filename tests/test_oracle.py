"""The CPU oracle against the reference's golden values (CPU only).

Pins oracle/crc32_oracle.c to: the reference tests' KATs (tests/fs.c:201-214),
zlib.crc32, the bit-at-a-time definition, the reference's compiled
deps/crc32/crc32.c (oracle/_ref, when built) and tests/golden/crc32_vectors.json.
"""
import zlib

import numpy as np
import pytest

from chunkio_amd import workloads as wl
from oracle import pyoracle as po

INIT = 0xFFFFFFFF


def kat_bytes(k, data400):
    if "hex" in k:
        return bytes.fromhex(k["hex"])
    return {"zero2_400kb_fs.c:209": b"\0\0" + data400, "400kb": data400,
            "zero2_5x400kb_cio_perf_file": b"\0\0" + data400 * 5}[k["name"]]


def test_reference_expectations(data400):
    # tests/fs.c:201-206 (empty chunk after sync) and :209-214 (after one 400 KB write)
    assert po.crc_update(INIT, b"\0\0") ^ INIT == 0x41D912FF
    assert po.crc_update(INIT, b"\0\0" + data400) ^ INIT == 0x103CFA67


def test_kats(golden, data400):
    for k in golden["kats"]:
        data = kat_bytes(k, data400)
        assert len(data) == k["len"]
        assert po.crc_update(INIT, data) == k["raw"], k["name"]
        assert zlib.crc32(data) == k["crc32"], k["name"]


def test_random_by_len(golden):
    g = golden["random_by_len"]
    for n in range(0, g["max_len"] + 1, 7):
        data = wl.gen_chunk(g["seed"], n, n)
        assert po.crc_update(INIT, data) == g["raw"][n], n


def test_seeded(golden):
    g = golden["seeded"]
    for v in g["vectors"]:
        data = wl.gen_chunk(g["data_seed"], v["len"], v["len"])
        assert po.crc_update(v["seed"], data) == v["raw"], v


def test_alignment_independent():
    data = wl.gen_chunk(7, 0, 5000)
    buf = np.zeros(5000 + 32, dtype=np.uint8)
    want = po.crc_bitwise(INIT, data)
    for mis in range(16):
        buf[mis:mis + 5000] = data
        assert po.crc_update(INIT, buf[mis:mis + 5000]) == want


def test_bitwise_definition():
    rng = np.random.default_rng(1)
    for n in [0, 1, 2, 7, 8, 9, 100, 1031]:
        data = rng.integers(0, 256, n, dtype=np.uint8)
        for seed in (0, INIT, 0x1234ABCD):
            assert po.crc_update(seed, data) == po.crc_bitwise(seed, data)


@pytest.mark.skipif(po.ref() is None, reason="oracle/_ref not built (no /root/reference)")
def test_against_compiled_reference():
    rng = np.random.default_rng(2)
    for n in list(range(0, 300)) + [4095, 4096, 4097, 65537]:
        data = rng.integers(0, 256, n, dtype=np.uint8)
        for seed in (0, INIT, 0xBE26ED00):
            assert po.crc_update(seed, data) == po.crc_update_ref(seed, data)


def test_shift_combine_identities():
    rng = np.random.default_rng(3)
    for na, nb in [(0, 0), (1, 0), (0, 5), (13, 29), (4096, 4032), (70000, 123457)]:
        a = rng.integers(0, 256, na, dtype=np.uint8)
        b = rng.integers(0, 256, nb, dtype=np.uint8)
        for seed in (0, INIT, 0x89ABCDEF):
            whole = po.crc_update(seed, np.concatenate([a, b]))
            # crc(s, A||B) = shift(crc(s, A), |B|) ^ crc(0, B)
            assert po.crc_shift(po.crc_update(seed, a), nb) ^ po.crc_update(0, b) == whole
            # shift(s, n) = crc(s, zeros(n))
            assert po.crc_shift(seed, nb) == po.crc_update(seed, np.zeros(nb, np.uint8))


def test_cfg_geometry(golden):
    import hashlib
    l3 = wl.cfg3_lens()
    g = golden["cfg3"]
    assert int(l3.sum()) == g["total_bytes"]
    assert hashlib.sha256(l3.astype("<u8").tobytes()).hexdigest() == g["lens_sha256"]
    assert l3.min() >= 4096 and l3.max() < 4 * 1024 * 1024
    assert (l3 % 4096 != 0).mean() > 0.99      # non-4K-multiple lengths present


def test_cfg2_first_chunks(golden):
    g = golden["cfg2"]
    got = po.crc_batch_chunks(g["seed"], wl.cfg2_lens(), idx=range(8))
    assert list(got) == g["first32"][:8]


def test_multithreaded_batch_timer_matches_single_thread():
    """oracle's crc_batch_time_mt (the bench's nproc-thread CPU figure) gives
    the same CRCs as the single-thread timer and the restatement."""
    import ctypes
    from chunkio_amd import workloads as wl
    lens = np.asarray([0, 1, 7, 4096, 70001, 409600] * 5, dtype=np.uint64)
    buf, offs = wl.host_batch(0x77, lens)
    lib = po.oracle()
    f = lib.oracle_crc_batch_time_mt
    f.restype = ctypes.c_double
    u64p = ctypes.POINTER(ctypes.c_uint64)
    f.argtypes = [ctypes.c_void_p, u64p, u64p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                  ctypes.POINTER(ctypes.c_uint32)]
    out = np.zeros(len(lens), np.uint32)
    offs = np.ascontiguousarray(offs, np.uint64)
    f(buf.ctypes.data, offs.ctypes.data_as(u64p), lens.ctypes.data_as(u64p), len(lens), 2, 4,
      out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    np.testing.assert_array_equal(out, po.crc_batch(buf, offs, lens))


def test_cfg5_full_digest_fixture(golden):
    """The cfg5 fixture (SHA-256 over all 1,024 digests) recomputed with
    hashlib from the generator: the GPU tests compare against this value."""
    import hashlib
    d = b"".join(hashlib.sha1(wl.gen_chunk(wl.CFG2_SEED, i, wl.CFG2_LEN).tobytes()).digest()
                 for i in range(wl.CFG2_N))
    assert hashlib.sha256(d).hexdigest() == golden["sha1"]["cfg5_sha256_of_digests"]
    assert [d[20 * i:20 * i + 20].hex() for i in range(8)] == golden["sha1"]["cfg2_first8"]


def test_cfg3_fixture_samples_and_digest_shape(golden):
    """cfg3's pinned samples recomputed with zlib (a second oracle beside the
    reference crc32.c that made them); the 65,536-CRC digest itself is checked
    on the GPU (test_cfg3_mixed_sizes_full), 39.7 GB being too much for the CPU suite."""
    import zlib
    g = golden["cfg3"]
    l3 = wl.cfg3_lens()
    for i, raw in list(zip(g["sample_idx"], g["sample_raw"]))[::8]:
        assert zlib.crc32(wl.gen_chunk(g["seed"], i, int(l3[i])).tobytes()) ^ 0xFFFFFFFF == raw
    assert len(g["sha256_of_raw_le"]) == 64


def test_weak_job_fixtures(golden):
    """The weak-job digests (bench.py --gpus N, N = 1..8) agree at N = 1 with
    the per-config fixtures made by the separate full-batch passes, cfg2's
    N = 2 job is recomputed here with zlib, and cfg3's lengths are a prefix-
    stable function of the chunk id (the N-GPU job is the first N x 65 536)."""
    import hashlib
    import zlib
    j = golden["weak_jobs"]
    assert j["cfg2"]["1"] == golden["cfg2"]["sha256_of_raw_le"]
    assert j["cfg3"]["1"] == golden["cfg3"]["sha256_of_raw_le"]
    assert j["sha1"]["1"] == golden["sha1"]["cfg5_sha256_of_digests"]
    for k in ("cfg2", "cfg4k", "cfg3", "sha1"):
        assert sorted(j[k], key=int) == [str(g) for g in range(1, 9)]
        assert len(set(j[k].values())) == 8
    c2 = np.asarray([zlib.crc32(wl.gen_chunk(wl.CFG2_SEED, i, wl.CFG2_LEN).tobytes()) ^ 0xFFFFFFFF
                     for i in range(2 * wl.CFG2_N)], np.uint32)
    assert hashlib.sha256(c2.astype("<u4").tobytes()).hexdigest() == j["cfg2"]["2"]
    np.testing.assert_array_equal(wl.cfg3_lens(8 * wl.CFG3_N)[: wl.CFG3_N], wl.cfg3_lens())
