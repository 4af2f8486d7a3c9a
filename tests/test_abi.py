"""C ABI of libchunkio_amd.so on the CPU: loads, exports every declared
symbol, and its host-side math (crc_update, shift, combine) matches the
oracle.  No GPU compute calls here."""
import ctypes
import os
import re

import numpy as np
import pytest

import chunkio_amd
from chunkio_amd import _lib
from oracle import pyoracle as po

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INIT = 0xFFFFFFFF


def declared_functions():
    names = set()
    for hdr in ("include/crc32/crc32.h", "include/chunkio_amd/cio_crc32_gpu.h",
                "include/chunkio_amd/cio_verify.h", "include/chunkio_amd/cio_sync.h",
                "include/chunkio_amd/cioa_chunk.h", "include/chunkio_amd/cio_sha1.h", "include/sha1/sha1.h"):
        text = open(os.path.join(ROOT, hdr)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^\s*(?!static|typedef|#)[A-Za-z_][\w\s\*]*?\b([a-z_][A-Za-z0-9_]*)\s*\(",
                             text, flags=re.M):
            names.add(m.group(1))
    return names


def test_library_loads_and_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    decl = declared_functions()
    assert "crc_update" in decl and "cio_crc32_plan_exec" in decl
    assert {"cio_sha1_hash", "cioa_SHA1_Update", "cioa_chunk_up_batch"} <= decl
    missing = [n for n in sorted(decl) if not hasattr(lib, n)]
    assert not missing, missing
    assert set(_lib.EXPORTS) >= decl, sorted(decl - set(_lib.EXPORTS))


def test_version_string():
    assert b"gfx950" in chunkio_amd.lib().cio_gpu_version()


@pytest.mark.parametrize("seed", [0, INIT, 0xBE26ED00])
def test_crc_update_matches_oracle(seed):
    rng = np.random.default_rng(11)
    buf = rng.integers(0, 256, 70000, dtype=np.uint8)
    for n in list(range(0, 80)) + [127, 128, 129, 4095, 4096, 4097, 65536 + 3]:
        for mis in (0, 1, 5, 15):
            chunk = buf[mis:mis + n]
            assert chunkio_amd.crc_update(seed, chunk) == po.crc_update(seed, chunk)


@pytest.mark.parametrize("mode", ["table", "clmul", "auto"])
def test_crc_update_host_paths(mode):
    """Every host path of the drop-in crc_update (slice-by-16 tables, 128-bit
    PCLMULQDQ folding, 512-bit VPCLMULQDQ folding; CIOA_HOST_CRC picks one
    per process) against the oracle at the fold boundaries, misaligned, and
    with seeds.  (Where the CPU lacks the instructions, the table path runs.)"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"""
import sys; sys.path.insert(0, {root!r})
import numpy as np, chunkio_amd as c
from oracle import pyoracle as po
rng = np.random.default_rng(3)
buf = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
lens = list(range(0, 300)) + [511, 512, 513, 1023, 1024, 1025, 1279, 1280, 1281, 4096, 65536 + 17, (3 << 20) - 31]
for n in lens:
    for mis in (0, 1, 7, 15):
        ch = buf[mis:mis + n]
        for s in (0, 0xFFFFFFFF, 0xBE26ED00):
            assert c.crc_update(s, ch) == po.crc_update(s, ch), (n, mis, s)
print("ok")
"""
    env = dict(os.environ, CIOA_HOST_CRC=mode, CIO_GPU_DIAG="1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr


WIDE_SEEDS_CODE = """
import sys; sys.path.insert(0, {root!r})
import numpy as np, chunkio_amd as c
from oracle import pyoracle as po
rng = np.random.default_rng(5)
raw = rng.integers(0, 256, 409600 + 64, dtype=np.uint8)
a0 = (-raw.ctypes.data) % 8                       # raw[a0:] is 8-byte aligned
seeds = [0x1FFFFFFFF, 0xFFFFFFFF12345678, 0xABCD00000000ABCD, 0xFFFFFFFFFFFFFFFF,
         0x0000000100000000, 0xFFFFFFFF, 0xBE26ED00, 0]
seeds += [int(s) for s in rng.integers(0, 2 ** 63, 4, dtype=np.int64) * 2 + 1]
lens = list(range(0, 18)) + [63, 64, 65, 1023, 1024, 4093, 409600]
ref = po.ref()
diff = n = 0
for s in seeds:
    for mis in range(8):
        for L in lens:
            ch = raw[a0 + mis:a0 + mis + L]
            assert ch.ctypes.data % 8 == mis or L == 0
            got, want = c.crc_update(s, ch), po.crc_update(s, ch)
            if ref is not None:
                r = po.crc_update_ref(s, ch)
                assert want == r, ("oracle vs _ref", hex(s), mis, L, hex(want), hex(r))
            diff += got != want
            n += 1
assert diff == 0, (diff, n)
print("ok", n, ref is not None)
"""


@pytest.mark.parametrize("mode", ["table", "clmul", "auto"])
def test_crc_update_wide_crc_t_states(mode):
    """crc_t is 8 bytes and deps/crc32 does not mask its input: a state with
    bits 32..63 set folds bits 32..39 into the first byte-wise step
    (crc32.c:343-348 / :384-386) and drops them on an 8-aligned word step
    (:366).  The drop-in crc_update (every host path), the oracle and the
    reference compiled unmodified (oracle/_ref) must agree on every such
    state, at misalignment 0..7 and lengths around every path switch."""
    import subprocess
    import sys
    code = WIDE_SEEDS_CODE.format(root=ROOT)
    env = dict(os.environ, CIOA_HOST_CRC=mode, CIO_GPU_DIAG="1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stderr[-3000:]


def test_wide_state_rule_restated_in_python():
    """The first-step rule, restated without any table library: one bitwise
    byte step on the full 64-bit state, then the ordinary 32-bit CRC."""
    def bitwise(c, data):
        for b in data:
            c ^= b
            for _ in range(8):
                c = (c >> 1) ^ (0xEDB88320 if c & 1 else 0)
        return c
    lib = ctypes.CDLL(_lib.LIB_PATH)
    f = lib.crc_update
    f.restype = ctypes.c_uint64
    f.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t]
    buf = (ctypes.c_uint8 * 64)(*range(1, 65))
    base = ctypes.addressof(buf)
    seed = 0xABCD005A0000ABCD     # bits 32..39 = 0x5A
    for start in range(16):
        p = base + start
        for L in (1, 5, 7, 8, 9, 40):
            data = bytes(buf[start:start + L])
            if (p % 8) or L < 8:
                t = seed ^ data[0]
                for _ in range(8):
                    t = (t >> 1) ^ (0xEDB88320 if t & 1 else 0)
                want = bitwise(t & 0xFFFFFFFF, data[1:])
            else:
                want = bitwise(seed & 0xFFFFFFFF, data)
            assert f(seed, p, L) == want, (start, L)


def test_crc_update_kats(data400):
    assert chunkio_amd.crc32(b"123456789") == 0xCBF43926
    assert chunkio_amd.crc32(b"\0\0") == 0x41D912FF
    assert chunkio_amd.crc32(b"\0\0" + data400) == 0x103CFA67
    assert chunkio_amd.crc32(b"\0\0" + data400 * 5) == 0x088740E7
    assert chunkio_amd.crc_update(INIT, b"") == INIT


def test_crc_t_is_8_bytes():
    # crc_t = uint_fast32_t is 8 bytes on LP64 Linux; cio_file.c:111 memcpy()s 8 bytes.
    assert ctypes.sizeof(ctypes.c_uint64) == 8
    lib = ctypes.CDLL(_lib.LIB_PATH)
    f = lib.crc_update
    f.restype = ctypes.c_uint64
    f.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t]
    # upper bits of the state are masked off, as in crc32.c:389
    assert f(0xFFFFFFFF00000000 | INIT, None, 0) == INIT


def test_shift_and_combine_match_oracle():
    rng = np.random.default_rng(12)
    for n in [0, 1, 3, 64, 4032, 4096, 409600, 2 ** 32 + 5, 2 ** 40]:
        s = int(rng.integers(0, 2 ** 32))
        assert chunkio_amd.crc32_shift(s, n) == po.crc_shift(s, n)
    a = rng.integers(0, 256, 1000, dtype=np.uint8)
    b = rng.integers(0, 256, 777, dtype=np.uint8)
    whole = po.crc_update(INIT, np.concatenate([a, b]))
    assert chunkio_amd.crc32_combine(po.crc_update(INIT, a), po.crc_update(0, b), len(b)) == whole


def test_sha1_entry_points_reject_null_pointers_without_a_gpu():
    """Argument checks run before any device call: a null descriptor or output
    pointer is CIO_ERROR with a message, not a fault (no GPU needed)."""
    lib = chunkio_amd.lib()
    buf = ctypes.create_string_buffer(64)
    assert lib.cio_sha1_batch_dev_async(None, None, None, None, 0, None) == 0   # empty batch: nothing to do
    assert lib.cio_sha1_batch_dev_async(buf, None, buf, buf, 1, None) == -1
    assert b"null pointer" in lib.cio_gpu_last_error()
    offs = (ctypes.c_uint64 * 1)(0)
    assert lib.cio_sha1_batch_dev(buf, offs, offs, None, 1, None) == -1
    assert b"null pointer" in lib.cio_gpu_last_error()


def test_plan_create_rejects_bad_arguments_without_a_gpu():
    """cio_crc32_plan_create checks its arguments before any device call:
    null arrays and 2^32 or more chunks are CIO_ERROR with a message."""
    lib = chunkio_amd.lib()
    h = ctypes.c_void_p()
    offs = (ctypes.c_uint64 * 1)(0)
    assert lib.cio_crc32_plan_create(None, offs, offs, 1) == -1
    assert b"null argument" in lib.cio_gpu_last_error()
    assert lib.cio_crc32_plan_create(ctypes.byref(h), None, offs, 1) == -1
    assert b"null argument" in lib.cio_gpu_last_error()
    assert lib.cio_crc32_plan_create(ctypes.byref(h), offs, offs, 1 << 32) == -1
    assert b"too many chunks" in lib.cio_gpu_last_error()
    assert not h.value


def test_library_shares_torchs_hip_runtime_when_loaded_first():
    """Loaded before torch, the library must bind torch's libamdhip64 (not a
    second copy from /opt/rocm): two HIP/HSA runtimes in one process leave the
    second to initialise with no device (seen on the GPU box as
    'hipGetDevice: no ROCm-capable device' in a lone test_chunkfile run)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"""
import sys; sys.path.insert(0, {root!r})
from chunkio_amd import _lib
_lib.lib()
assert "torch" not in sys.modules
hip = sorted({{l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l}})
import torch
hip2 = sorted({{l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l}})
print(len(hip), len(hip2), hip2[0].startswith(__import__("os").path.dirname(torch.__file__)))
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["1", "1", "True"], r.stdout


def test_hip_runtime_override_system():
    """CIOA_HIP_RUNTIME=system keeps the library on /opt/rocm's libamdhip64
    (one runtime as long as torch is not loaded into the same process)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"""
import sys; sys.path.insert(0, {root!r})
from chunkio_amd import _lib
_lib.lib()
hip = sorted({{l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l}})
print(len(hip), hip[0].startswith("/opt/rocm"), _lib._hip_runtime is None)
"""
    env = dict(os.environ, CIOA_HIP_RUNTIME="system")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["1", "True", "True"], r.stdout


def test_hip_runtime_pin_checks_soname(tmp_path, monkeypatch):
    """torch's libamdhip64 is pinned only when its SONAME is the one
    libchunkio_amd.so links (DT_NEEDED); a mismatching file is left alone with
    a warning naming both."""
    from chunkio_amd import _lib
    soname, _ = _lib._elf_dynamic_strings(_lib.LIB_PATH)
    _, needed = _lib._elf_dynamic_strings(_lib.LIB_PATH)
    assert any(x.startswith("libamdhip64.so") for x in needed), needed
    assert _lib._elf_dynamic_strings(str(tmp_path / "missing.so")) == (None, [])
    (tmp_path / "not_elf.so").write_bytes(b"not an elf file")
    assert _lib._elf_dynamic_strings(str(tmp_path / "not_elf.so")) == (None, [])
    # a torch whose runtime is another major version: no pin, a warning
    real = _lib._elf_dynamic_strings

    def fake(path):
        if path.endswith("libamdhip64.so"):
            return "libamdhip64.so.99", []
        return real(path)
    monkeypatch.setattr(_lib, "_elf_dynamic_strings", fake)
    monkeypatch.delenv("CIOA_HIP_RUNTIME", raising=False)
    import sys
    had_torch = sys.modules.pop("torch", None)
    try:
        import importlib.util
        if importlib.util.find_spec("torch") is None:
            pytest.skip("torch not installed")
        with pytest.warns(UserWarning, match="not pinning"):
            assert _lib._pin_hip_runtime() is None
    finally:
        if had_torch is not None:
            sys.modules["torch"] = had_torch
