"""The host CRC batch (cio_crc32_batch_cpu / _fd_cpu, crc_cpu_batch.c) and the
chunk layer's route between it and the GPU (crc_route.c).  CPU only: the host
batch is the library's crc_update spread over a thread pool, checked here
against the oracle (the reference's crc32.c restated, oracle/) bit for bit."""
import ctypes
import os

import numpy as np
import pytest

import chunkio_amd as cio
from chunkio_amd import _lib
from chunkio_amd import workloads as wl
from oracle import pyoracle as po

INIT = 0xFFFFFFFF


def _batch(seed, lens):
    lens = np.asarray(lens, dtype=np.uint64)
    buf, offs = wl.host_batch(seed, lens)
    return buf, offs, lens


@pytest.mark.parametrize("threads", [1, 2, 3, 8, 16])
def test_cpu_batch_matches_oracle(threads):
    # empty, tiny, piece-boundary (1 MiB) and multi-piece chunks, interleaved
    lens = [0, 1, 7, 4096, 409600, (1 << 20) - 1, 1 << 20, (1 << 20) + 1, 3 * (1 << 20) + 5, 0, 12345] * 3
    buf, offs, lens = _batch(0xC0FFEE, lens)
    got = cio.crc32_batch_cpu_packed(buf, offs, lens, threads=threads)
    np.testing.assert_array_equal(got, po.crc_batch(buf, offs, lens))


@pytest.mark.parametrize("threads", [1, 4])
def test_cpu_batch_seeds(threads):
    lens = np.asarray([0, 3, 5000, 2 * (1 << 20) + 77, 64], np.uint64)
    buf, offs, lens = _batch(0xABC, lens)
    seeds = np.asarray([0, 0xBE26ED00, 0x12345678, 0xDEADBEEF, INIT], np.uint32)
    got = cio.crc32_batch_cpu_packed(buf, offs, lens, seeds=seeds, threads=threads)
    want = [po.crc_update(int(s), buf[int(o):int(o + n)]) for s, o, n in zip(seeds, offs, lens)]
    np.testing.assert_array_equal(got, np.asarray(want, np.uint32))


def test_cpu_batch_one_large_chunk_uses_pieces():
    """A single 9 MiB + 3 chunk at a misaligned offset: 10 pieces folded with
    cio_crc32_combine must equal one crc_update over the whole chunk."""
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, 9 * (1 << 20) + 3 + 5, dtype=np.uint8)
    offs = np.asarray([5], np.uint64)
    lens = np.asarray([9 * (1 << 20) + 3], np.uint64)
    for t in (1, 2, 7, 16):
        got = cio.crc32_batch_cpu_packed(data, offs, lens, threads=t)
        assert int(got[0]) == po.crc_update(INIT, data[5:])


def test_cpu_batch_many_small_chunks_grouped():
    lens = np.full(20000, 100, np.uint64)
    lens[::7] = 0
    buf, offs, lens = _batch(0x77, lens)
    got = cio.crc32_batch_cpu_packed(buf, offs, lens, threads=16)
    np.testing.assert_array_equal(got, po.crc_batch(buf, offs, lens))


def test_cpu_batch_repeated_calls_and_thread_growth():
    """The persistent pool: calls with growing and shrinking thread counts
    (workers started for one call join it; idle ones sit out)."""
    buf, offs, lens = _batch(0x99, [300000] * 40)
    want = po.crc_batch(buf, offs, lens)
    for t in (2, 5, 3, 16, 1, 9, 16, 2):
        np.testing.assert_array_equal(cio.crc32_batch_cpu_packed(buf, offs, lens, threads=t), want)


def test_cpu_batch_concurrent_callers():
    import threading
    buf, offs, lens = _batch(0x31, [700000] * 16)
    want = po.crc_batch(buf, offs, lens)
    errs = []

    def run(t):
        try:
            for _ in range(5):
                np.testing.assert_array_equal(cio.crc32_batch_cpu_packed(buf, offs, lens, threads=t), want)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=run, args=(t,)) for t in (4, 8, 1, 16)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs


def _fd_cpu(fds, foffs, lens, threads):
    n = len(lens)
    P = ctypes.POINTER
    fds_a = (ctypes.c_int * max(n, 1))(*fds)
    fo = np.ascontiguousarray(foffs, np.uint64)
    ln = np.ascontiguousarray(lens, np.uint64)
    out = np.zeros(max(n, 1), np.uint32)
    rc = cio.lib().cio_crc32_batch_fd_cpu(fds_a, fo.ctypes.data_as(P(ctypes.c_uint64)),
                                          ln.ctypes.data_as(P(ctypes.c_size_t)), None,
                                          out.ctypes.data_as(P(ctypes.c_uint32)), n, threads)
    return rc, out[:n]


@pytest.mark.parametrize("threads", [1, 6])
def test_fd_cpu_batch(tmp_path, threads):
    rng = np.random.default_rng(11)
    paths, fds, foffs, lens, want = [], [], [], [], []
    for i, n in enumerate([0, 10, 1 << 20, 2_500_001, 409600]):
        data = rng.integers(0, 256, n + 22, dtype=np.uint8)
        p = tmp_path / f"c{i}"
        p.write_bytes(data.tobytes())
        paths.append(p)
        fds.append(os.open(p, os.O_RDONLY))
        foffs.append(22)
        lens.append(n)
        want.append(po.crc_update(INIT, data[22:]))
    try:
        rc, got = _fd_cpu(fds, foffs, lens, threads)
        assert rc == 0
        np.testing.assert_array_equal(got, np.asarray(want, np.uint32))
        # a range past the end of its file is a short read: CIO_ERROR
        rc, _ = _fd_cpu(fds, foffs, [lens[0], lens[1] + 5, lens[2], lens[3], lens[4]], threads)
        assert rc == -1
        assert b"short read" in cio.lib().cio_gpu_last_error()
    finally:
        for fd in fds:
            os.close(fd)


def test_route_threshold_follows_host_threads():
    """cio_crc32_cpu_max(): the cost model's crossover -- ~17 MB with one host
    thread, inside the slower MI355X box's measured crossover (host faster
    at 13.1 MB, GPU faster at 26.2 MB: profiles/r04/route_batch_r04d.json)
    and below the faster box's (52-105 MB), everything on the host with two
    or more (the host's DRAM rate beats one PCIe link); an explicit
    threshold overrides it."""
    lib = cio.lib()
    if os.environ.get("CIOA_CPU_CRC_MAX") or os.environ.get("CIOA_HOST_CRC_THREADS"):
        pytest.skip("routing environment set by the caller")
    before_max, before_t = cio.route()
    model_max = cio.route(reset=True)[0]
    try:
        assert cio.host_threads(1) == 1
        one = lib.cio_crc32_cpu_max()
        import json
        rows = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                           "profiles", "r04", "route_batch_r04d.json")))["rows"]
        host_won = max(r["bytes"] for r in rows if r["winner_1t"] == "cpu")
        gpu_won = min(r["bytes"] for r in rows if r["winner_1t"] == "gpu")
        assert host_won <= one < gpu_won, (host_won, one, gpu_won)
        assert cio.host_threads(16) == 16
        assert lib.cio_crc32_cpu_max() == ctypes.c_size_t(-1).value
        assert cio.host_threads(0) == 1          # clamped
        assert cio.host_threads(1000) == 64
        # an explicit threshold overrides the model, reset drops it again
        assert cio.route(cpu_max=12345)[0] == 12345
        assert cio.route(reset=True) == (model_max, 1)
    finally:
        cio.route(reset=True)
        if before_max != model_max:
            cio.route(cpu_max=before_max)
        if before_t != 1:
            cio.route(threads=before_t)


def test_split_point_sizing_model():
    """crc_route.c's split sizing for a batch the threshold sends to the GPU
    (no device needed): the host takes the largest suffix of whole chunks
    within B_host = (F + B / r_gpu) / (1 / r_host + 1 / r_gpu) at the model's
    rates; nothing is split when the GPU's share would be under 32 MB, when the
    split route is off, or when an explicit threshold picks the engine."""
    lib = ctypes.CDLL(_lib.LIB_PATH)
    f = lib.cioa_debug_split_point
    f.restype = ctypes.c_size_t
    f.argtypes = [ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    if os.environ.get("CIOA_CPU_CRC_MAX") or os.environ.get("CIOA_SPLIT_ROUTE") or os.environ.get("CIOA_HOST_CRC_THREADS"):
        pytest.skip("routing environment set by the caller")

    def point(lens, fd=1, ndev=1):
        arr = (ctypes.c_size_t * len(lens))(*lens)
        return int(f(arr, len(lens), ndev, fd, 1))

    try:
        cio.route(reset=True, threads=1)
        cio.split_rates(forget=True)
        lens = [2048002] * 1000                            # the verify leg's 1000 perf files
        B = float(sum(lens))
        for fd, r_host in ((1, 22.0), (0, 36.0)):
            for ndev in (1, 2):
                r_gpu = 54.7 * ndev
                b_host = (163.5e-6 + B / (r_gpu * 1e9)) / (1 / (r_host * 1e9) + 1 / (r_gpu * 1e9))
                k = point(lens, fd, ndev)
                assert sum(lens[k:]) <= b_host < sum(lens[k - 1:]), (fd, ndev, k)
        assert point([2048002] * 12) == 12                 # 24.6 MB: the GPU's share would be < 32 MB
        cio.route(split=False)
        assert point(lens) == len(lens)
        cio.route(reset=True, cpu_max=1)                   # explicit threshold: the GPU alone
        assert point(lens) == len(lens)
        cio.route(split=True)                              # ... unless the split is turned on too
        assert point(lens) < len(lens)
        cio.route(reset=True, cpu_max=1, split="force")    # forced: even 2 chunks of 1 byte
        assert point([1, 1]) == 1
    finally:
        cio.route(reset=True)
        cio.split_rates(forget=True)


def test_split_route_recovers_from_a_low_learned_gpu_rate():
    """a GPU rate learned too low kept a host-routed batch off the
    split route for good (no split, so no new sample).  Each such decision now
    moves the learned rate a tenth of the way back to the model (54.7 GB/s),
    so the route tries a split again after a few batches; a rate at or above
    the model is left alone."""
    lib = ctypes.CDLL(_lib.LIB_PATH)
    f = lib.cioa_debug_split_point
    f.restype = ctypes.c_size_t
    f.argtypes = [ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    setr = lib.cioa_debug_split_set_gpu_rate
    setr.argtypes = [ctypes.c_int, ctypes.c_double]
    if os.environ.get("CIOA_CPU_CRC_MAX") or os.environ.get("CIOA_SPLIT_ROUTE") or os.environ.get("CIOA_HOST_CRC_THREADS"):
        pytest.skip("routing environment set by the caller")
    lens = (ctypes.c_size_t * 200)(*([2048002] * 200))
    try:
        cio.route(reset=True, threads=4)                  # host-routed: 4 x 22 GB/s from files
        cio.split_rates(forget=True)
        setr(1, 10.0)                                     # learned far too low (cold first split)
        assert cio.split_rates()["gpu_fd"] == pytest.approx(10.0)
        seen = []
        for _ in range(40):
            f(lens, 200, 1, 1, 0)                         # host-routed, fd batch
            seen.append(cio.split_rates()["gpu_fd"])
        assert seen[0] == pytest.approx(10.0 + 0.1 * (54.7 - 10.0))
        assert all(b >= a for a, b in zip(seen, seen[1:]))
        assert 88.0 < 3 * seen[-1] <= 3 * 54.7           # recovered: the split is considered again
        setr(1, 60.0)                                     # at or above the model: untouched
        f(lens, 200, 1, 1, 0)
        assert cio.split_rates()["gpu_fd"] == pytest.approx(60.0)
    finally:
        cio.route(reset=True)
        cio.split_rates(forget=True)


def test_library_unload_stops_the_host_crc_pool():
    """The host CRC pool's detached workers run the library's code: dlclose
    (and exit) tells them to leave first (crc_cpu_batch.c pool_stop), so a
    process that unloads the library after an 8-thread batch keeps running."""
    import subprocess
    import sys
    code = f"""
import ctypes, _ctypes, time, numpy as np
lib = ctypes.CDLL({_lib.LIB_PATH!r}, mode=ctypes.RTLD_LOCAL)
n = 64
bufs = [np.full(1 << 20, i, np.uint8) for i in range(n)]
ptrs = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
lens = (ctypes.c_size_t * n)(*[b.size for b in bufs])
out = (ctypes.c_uint32 * n)()
assert lib.cio_crc32_batch_cpu(ptrs, lens, None, out, n, 8) == 0
h = lib._handle
del lib
_ctypes.dlclose(h)
time.sleep(0.5)
print("alive")
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "alive", (r.returncode, r.stderr[-2000:])


def test_host_paths_past_4gib():
    """Host CRC over 4 GiB + 5 bytes (lengths and offsets past 32 bits): the
    drop-in crc_update (crc32.c:337 takes a size_t length) and the host batch
    pool on 1 and 4 threads, against zlib.  The data repeats every 1,000,003
    bytes, so a 32-bit offset wrap would read different bytes."""
    import zlib
    n = (4 << 30) + 5
    block = np.random.default_rng(44).integers(0, 256, 1_000_003, dtype=np.uint8)
    buf = np.resize(block, n + 64)
    want_full = zlib.crc32(memoryview(buf[3:3 + n])) ^ 0xFFFFFFFF
    assert cio.crc_update(cio.crc_init(), memoryview(buf[3:3 + n])) == want_full
    offs = np.asarray([0, 3, n + 7], np.uint64)
    lens = np.asarray([3, n, 50], np.uint64)
    want = [zlib.crc32(memoryview(buf[int(o):int(o + ln)])) ^ 0xFFFFFFFF for o, ln in zip(offs, lens)]
    for t in (1, 4):
        got = cio.crc32_batch_cpu_packed(buf, offs, lens, threads=t)
        assert [int(x) for x in got] == want, t
