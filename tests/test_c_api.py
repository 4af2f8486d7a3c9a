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


def test_make_install_and_link_from_the_prefix(tmp_path):
    """`make install PREFIX=...` lays out the library, the public headers and a
    pkg-config file; a C program built only against that prefix gets the
    reference's check value from crc_update and FIPS 180-4's "abc" digest from
    cio_sha1_hash."""
    prefix = tmp_path / "prefix"
    rc, out = _run(["make", "-s", "-C", ROOT, "install", f"PREFIX={prefix}"])
    assert rc == 0, out
    pc = (prefix / "lib" / "pkgconfig" / "chunkio_amd.pc").read_text()
    assert "-lchunkio_amd" in pc and f"prefix={prefix}" in pc
    for h in ("crc32/crc32.h", "sha1/sha1.h", "chunkio_amd/cio_sha1.h", "chunkio_amd/cio_sha1_state.h",
              "chunkio_amd/cio_crc32_gpu.h", "chunkio_amd/cioa_chunk.h"):
        assert (prefix / "include" / h).exists(), h
    src = tmp_path / "t.c"
    src.write_text(
        '#include <stdio.h>\n#include <string.h>\n#include <crc32/crc32.h>\n#include <chunkio_amd/cio_sha1.h>\n'
        'int main(void) { crc_t c = crc_finalize(crc_update(crc_init(), "123456789", 9));\n'
        '  unsigned char md[20]; char hex[41]; cio_sha1_hash("abc", 3, md, NULL); cio_sha1_to_hex(md, hex);\n'
        '  printf("%08lx %s\\n", (unsigned long) c, hex); return 0; }\n')
    exe = tmp_path / "t"
    rc, out = _run(["gcc", "-o", str(exe), str(src), f"-I{prefix}/include", f"-L{prefix}/lib", "-lchunkio_amd",
                    f"-Wl,-rpath,{prefix}/lib"])
    assert rc == 0, out
    rc, out = _run([str(exe)])
    assert rc == 0 and out.strip() == "cbf43926 a9993e364706816aba3e25717850c26c9cd0d89d", out


@pytest.mark.parametrize("lang", ["c", "c++"])
def test_public_headers_compile_alone_and_together(tmp_path, lang):
    """Every public header compiles on its own and all of them together, as C
    (gnu11) and as C++ (c++17, extern "C" linkage): a caller can include any
    subset in any order."""
    import glob
    hdrs = sorted(os.path.relpath(h, os.path.join(ROOT, "include"))
                  for h in glob.glob(os.path.join(ROOT, "include", "*", "*.h")))
    assert "sha1/sha1.h" in hdrs and "crc32/crc32.h" in hdrs
    comp, std, ext = ("gcc", "-std=gnu11", "c") if lang == "c" else ("g++", "-std=c++17", "cpp")
    for i, group in enumerate([[h] for h in hdrs] + [hdrs, hdrs[::-1]]):
        src = tmp_path / f"t{i}.{ext}"
        src.write_text("".join(f"#include <{h}>\n" for h in group) + "int main(void) { return 0; }\n")
        rc, out = _run([comp, std, "-Wall", "-Wextra", "-Werror", "-fsyntax-only", f"-I{ROOT}/include", str(src)])
        assert rc == 0, (group, out)
