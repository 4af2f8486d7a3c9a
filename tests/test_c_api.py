"""C callers of the public headers (tests/c/, built by `make ctests`).

test_crc32_dropin: the drop-in boundary from C -- chunkio's own
include/chunkio/cio_crc32.h macros (unmodified, where /root/reference exists
at build time) over include/crc32/crc32.h, linked against libchunkio_amd.so,
replaying the reference's call sites and golden values.  CPU only.

test_chunk_api: the reference's tests/fs.c and tests/metadata_update.c
replayed through include/chunkio_amd/cioa_chunk.h, plus transactions, trim,
full sync, batched scan with CIO_DELETE_IRRECOVERABLE and deferred/immediate
byte identity; in the reference's per-write order (immediate) and with the
CRC deferred to batched GPU syncs (deferred).  Verifies run on the GPU
(CIOA_CPU_CRC_MAX=0) under -m gpu, and on the host CRC route in the CPU
suite.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "c", "bin")
DATA = os.path.join(ROOT, "tests", "golden", "400kb.txt")


def _bin(name):
    p = os.path.join(BIN, name)
    if not os.path.exists(p):
        pytest.fail(f"{p} is not built: run `make ctests` (or __graft_entry__.build())")
    return p


def _run(args, timeout=600, env=None):
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout,
                       env=None if env is None else {**os.environ, **env})
    return r.returncode, r.stdout + r.stderr


def test_dropin_boundary_from_c():
    rc, out = _run([_bin("test_crc32_dropin"), DATA])
    assert rc == 0, out


def test_dropin_boundary_reference_header():
    p = os.path.join(BIN, "test_crc32_dropin_ref")
    if not os.path.exists(p):
        pytest.skip("built only where /root/reference exists (this container)")
    rc, out = _run([p, DATA])
    assert rc == 0 and "reference include/chunkio/cio_crc32.h" in out, out


@pytest.mark.parametrize("name", ["fs_deep_hierachy", "issue_51", "fs_checksum"])
def test_chunk_api_cpu_paths(tmp_path, name):
    """Reference tests whose chunks never re-verify an existing file: no GPU call."""
    rc, out = _run([_bin("test_chunk_api"), DATA, str(tmp_path), "immediate", name])
    assert rc == 0 and f"{name}" in out and "0 failed" in out, out


@pytest.mark.gpu
def test_chunk_api_reference_tests_immediate_and_deferred(cuda, tmp_path):
    """Every verify, recompute and deferred sync on the GPU route
    (CIOA_CPU_CRC_MAX=0: no batch is small enough for the host CRC)."""
    for mode in ("immediate", "deferred"):
        rc, out = _run([_bin("test_chunk_api"), DATA, str(tmp_path), mode], env={"CIOA_CPU_CRC_MAX": "0"})
        print(out)
        assert rc == 0, out


@pytest.mark.parametrize("threads", ["1", "8"])
def test_chunk_api_reference_tests_host_route(tmp_path, threads):
    """The same C replay with every chunk-layer CRC on the library's host
    crc_update (CIOA_CPU_CRC_MAX huge, crc_route.c), on the calling thread and
    on the 8-thread host pool (CIOA_HOST_CRC_THREADS): the chunk API's
    semantics do not depend on where the CRC runs.  (The deferred run
    compares its identity corpus with the immediate run's files.)"""
    for mode in ("immediate", "deferred"):
        rc, out = _run([_bin("test_chunk_api"), DATA, str(tmp_path), mode],
                       env={"CIOA_CPU_CRC_MAX": str(1 << 62), "CIOA_HOST_CRC_THREADS": threads})
        assert rc == 0 and "0 failed" in out, out


@pytest.mark.gpu
def test_multi_device_host_batches_from_c(cuda, tmp_path):
    """tests/c/test_multi.c: cio_crc32_batch_host_multi / _fd_multi /
    cio_crc32_split_host_multi over 1-4 device entries (each with its own host
    thread, pipeline and stream) and 6 concurrent callers sharing the
    per-device pipeline pool, every CRC against a bit-serial CRC-32 written in
    the test."""
    rc, out = _run([_bin("test_multi"), str(tmp_path)], timeout=300)
    print(out)
    assert rc == 0 and "0 failed" in out, out
