"""chunkio's SHA-1 interface (include/chunkio_amd/cio_sha1.h, include/sha1/sha1.h)
against OpenSSL itself.

The reference wraps an un-vendored <sha1/sha1.h> whose API is OpenSSL's
(src/cio_sha1.c:26-68, include/chunkio/cio_sha1.h:25-34): struct cio_sha1 holds
a SHA_CTX, and cio_sha1_hash copies the pre-Final SHA_CTX into `state`
(:52-54).  The oracle is OpenSSL's libcrypto in this container, called through
ctypes: every context byte the library leaves (after Init, each Update, Final,
and cio_sha1_hash's exported state) must equal what SHA1_Init / SHA1_Update /
SHA1_Final leave in an OpenSSL SHA_CTX at the same split points, on both host
block paths (SHA extensions and portable).  The reference's own cio_sha1.h and
cio_sha1.c, compiled unmodified against include/sha1/sha1.h, are run the same
way (tests/c/bin/test_sha1_ref, where /root/reference exists).  CPU only.
"""
import ctypes
import ctypes.util
import hashlib
import os
import subprocess

import numpy as np
import pytest

import chunkio_amd as cio
from chunkio_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "c", "bin")
DATA = os.path.join(ROOT, "tests", "golden", "400kb.txt")
SPLIT_LENS = (0, 1, 3, 55, 56, 57, 63, 64, 65, 119, 127, 128, 129, 1000, 4099, 65536)


def _crypto():
    name = ctypes.util.find_library("crypto")
    if not name:
        pytest.skip("OpenSSL libcrypto is not installed here")
    c = ctypes.CDLL(name)
    for fn in ("SHA1_Init", "SHA1_Update", "SHA1_Final"):
        if not hasattr(c, fn):
            pytest.skip(f"libcrypto lacks {fn}")
    c.SHA1_Init.argtypes = [ctypes.c_void_p]
    c.SHA1_Update.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    c.SHA1_Final.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    return c


class OsslCtx:
    """An OpenSSL SHA_CTX in a 96-byte buffer (sizeof(SHA_CTX) on LP64)."""

    def __init__(self, c, state=None):
        self.c = c
        self.buf = ctypes.create_string_buffer(96)
        if state is None:
            assert c.SHA1_Init(self.buf) == 1
        else:
            ctypes.memmove(self.buf, bytes(state), 96)

    def update(self, b):
        assert self.c.SHA1_Update(self.buf, b, len(b)) == 1

    def final(self):
        md = ctypes.create_string_buffer(20)
        assert self.c.SHA1_Final(md, self.buf) == 1
        return md.raw

    @property
    def state(self):
        return self.buf.raw


def _cases(seed, n):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        k = int(rng.integers(1, 6))
        out.append([int(rng.choice(SPLIT_LENS)) if rng.random() < 0.6 else int(rng.integers(0, 9000))
                    for _ in range(k)])
    return rng, out


@pytest.fixture(params=["shani", "portable"])
def host_path(request):
    lib = _lib.lib()
    lib.cioa_host_sha1_path.restype = ctypes.c_char_p
    lib.cioa_debug_host_sha1_pin(1 if request.param == "portable" else 0)
    got = lib.cioa_host_sha1_path().decode()
    if request.param == "shani" and got != "shani":
        lib.cioa_debug_host_sha1_pin(0)
        pytest.skip("this CPU has no SHA extensions")
    yield got
    lib.cioa_debug_host_sha1_pin(0)


def test_context_bytes_equal_openssl(host_path):
    """Random messages at random split points (block boundaries, 55/56/63/64
    padding edges, empty updates): the 96 context bytes after SHA1_Init, after
    every SHA1_Update and after SHA1_Final equal OpenSSL's; the digests equal
    hashlib's."""
    c = _crypto()
    rng, cases = _cases(61, 400)
    for pieces in cases:
        ours, ref = cio.Sha1(), OsslCtx(c)
        assert ours.state == ref.state
        msg = b""
        for ln in pieces:
            d = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
            ours.update(d)
            ref.update(d)
            msg += d
            assert ours.state == ref.state, (pieces, len(msg))
        md = ours.final()
        assert md == ref.final() == hashlib.sha1(msg).digest()
        assert ours.state == ref.state, ("after final", pieces)


def test_contexts_move_between_openssl_and_the_library(host_path):
    """A context OpenSSL built continues in the library and vice versa, at any
    split: the digest is the whole message's, and the bytes match at every
    hand-over."""
    c = _crypto()
    rng, cases = _cases(62, 200)
    for i, pieces in enumerate(cases):
        chunks = [rng.integers(0, 256, ln, dtype=np.uint8).tobytes() for ln in pieces]
        ref = OsslCtx(c)
        ours = cio.Sha1()
        for k, d in enumerate(chunks):
            # alternate the engine carrying the context, handing over the 96 bytes
            if (i + k) % 2:
                ours = cio.Sha1(ref.state)
                ours.update(d)
                ref = OsslCtx(c, ours.state)
            else:
                ref = OsslCtx(c, ours.state)
                ref.update(d)
                ours = cio.Sha1(ref.state)
        whole = hashlib.sha1(b"".join(chunks)).digest()
        assert ours.state == ref.state
        assert ours.final() == whole and ref.final() == whole


def test_cio_sha1_hash_state_and_hex(host_path):
    """cio_sha1_hash: digest, and `state` = OpenSSL's context after
    SHA1_Init + SHA1_Update of the message (before Final), which continues to
    the digest of a longer message; cio_sha1_to_hex is %02x per byte
    (src/cio_sha1.c:59-68)."""
    c = _crypto()
    rng = np.random.default_rng(63)
    for ln in list(SPLIT_LENS) + [409600]:
        msg = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
        md, st = cio.sha1_hash(msg, want_state=True)
        ref = OsslCtx(c)
        ref.update(msg)
        assert st == ref.state, ln
        assert md == hashlib.sha1(msg).digest()
        assert cio.sha1_hash(msg) == md
        assert cio.sha1_to_hex(md) == md.hex()
        more = b"tail" * (ln % 7)
        cont = cio.Sha1(st)
        cont.update(more)
        assert cont.final() == hashlib.sha1(msg + more).digest()


def test_bit_count_carries_past_2_32_bits():
    """Nl/Nh: a context whose bit count sits just below 2^32 (built by
    OpenSSL from 512 MiB - 3 bytes) carries into Nh on the next update exactly
    as OpenSSL's does.  (One 512 MiB pass each, ~0.5 s.)"""
    c = _crypto()
    big = np.frombuffer(np.random.default_rng(64).bytes(1 << 20), np.uint8)
    ref, ours = OsslCtx(c), cio.Sha1()
    for _ in range(511):
        ref.update(big.tobytes())
        ours.update(big.tobytes())
    tail = big[:(1 << 20) - 3].tobytes()
    ref.update(tail)
    ours.update(tail)
    assert ours.state == ref.state
    assert int.from_bytes(ref.state[24:28], "little") == 0           # Nh still 0
    ref.update(b"abcdefgh")
    ours.update(b"abcdefgh")
    assert ours.state == ref.state
    assert int.from_bytes(ref.state[24:28], "little") == 1           # carried
    assert ours.final() == ref.final()


def _run_c(binary, cases):
    args = [binary, DATA] + [f"{off}:{','.join(map(str, pieces))}" for off, pieces in cases]
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


@pytest.mark.parametrize("name", ["test_sha1", "test_sha1_ref"])
def test_c_callers_against_openssl(name):
    """From C: the library's cio_sha1_* (test_sha1) and the reference's own
    cio_sha1.h + cio_sha1.c compiled unmodified against include/sha1/sha1.h
    (test_sha1_ref): every context dump, digest and hex string equals what
    OpenSSL gives for the same calls."""
    p = os.path.join(BIN, name)
    if not os.path.exists(p):
        if name == "test_sha1_ref":
            pytest.skip("built only where /root/reference exists (this container)")
        pytest.fail(f"{p} is not built: run `make ctests`")
    c = _crypto()
    data = open(DATA, "rb").read()
    rng, plans = _cases(65, 40)
    cases = []
    for pieces in plans:
        total = sum(pieces)
        off = int(rng.integers(0, len(data) - total)) if total < len(data) else 0
        cases.append((off, pieces))
    cases.append((0, [len(data)]))
    out = _run_c(p, cases).splitlines()
    assert "sizeof(struct cio_sha1) 96" in out
    if name == "test_sha1_ref":
        assert "reference include/chunkio/cio_sha1.h + src/cio_sha1.c" in out
    lines = iter([ln for ln in out if ln.split(" ")[0] in ("case", "ctx", "md", "hash", "hex")])
    for off, pieces in cases:
        assert next(lines).startswith("case")
        ref = OsslCtx(c)
        assert next(lines) == "ctx " + ref.state.hex()
        pos = off
        for ln in pieces:
            ref.update(data[pos:pos + ln])
            pos += ln
            assert next(lines) == "ctx " + ref.state.hex()
        md = ref.final()
        assert next(lines) == f"md {md.hex()} {ref.state.hex()}"
        pre = OsslCtx(c)
        pre.update(data[off:pos])
        assert next(lines) == f"hash {md.hex()} {pre.state.hex()}"
        assert next(lines) == f"hex {md.hex()}"


def test_path_pins_need_the_diag_gate():
    """CIOA_HOST_SHA1=portable (an A/B pin) is ignored unless CIO_GPU_DIAG=1
    is set too: a stray variable cannot move a deployment off the SHA
    extensions.  (The GPU-side switches: test_gpu_crc.py's
    test_stray_switches_without_the_gate_change_nothing.)"""
    import sys
    code = ("import ctypes; from chunkio_amd import _lib; l = _lib.lib(); "
            "l.cioa_host_sha1_path.restype = ctypes.c_char_p; print(l.cioa_host_sha1_path().decode())")
    base = {k: v for k, v in os.environ.items() if k not in ("CIO_GPU_DIAG", "CIOA_HOST_SHA1")}
    run = lambda env: subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                                     env=env, cwd=ROOT).stdout.strip()
    best = run(base)
    assert run(dict(base, CIOA_HOST_SHA1="portable")) == best
    assert run(dict(base, CIOA_HOST_SHA1="portable", CIO_GPU_DIAG="1")) == "portable"


def test_context_oracle_pinned_to_openssl():
    """oracle/sha1_ctx.py (a pure-Python restatement of OpenSSL's SHA_CTX
    evolution, test infrastructure) gives OpenSSL's context bytes after every
    Init / Update / Final and hashlib's digests; the library agrees with both."""
    from oracle.sha1_ctx import Sha1Ctx
    c = _crypto()
    rng, cases = _cases(66, 120)
    for pieces in cases:
        o, ref, lib = Sha1Ctx(), OsslCtx(c), cio.Sha1()
        assert o.raw() == ref.state
        msg = b""
        for ln in pieces:
            d = rng.integers(0, 256, min(ln, 5000), dtype=np.uint8).tobytes()
            o.update(d)
            ref.update(d)
            lib.update(d)
            msg += d
            assert o.raw() == ref.state == lib.state, (pieces, len(msg))
        md = o.final()
        assert md == ref.final() == lib.final() == hashlib.sha1(msg).digest()
        assert o.raw() == ref.state == lib.state
        assert Sha1Ctx(ref.state).raw() == ref.state       # parse / serialise round trip


def _ctx_vectors():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "sha1_ctx_vectors.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("engine", ["library", "oracle"])
def test_context_bytes_against_openssl_fixtures(engine, host_path):
    """tests/golden/sha1_ctx_vectors.json: the SHA_CTX bytes libcrypto left
    after every piece and after Final (make_sha1_ctx.py), needing no OpenSSL
    at test time: the library's host SHA-1 (both block paths) and the
    context oracle reproduce every one."""
    from chunkio_amd import workloads as wl
    from oracle.sha1_ctx import Sha1Ctx
    g = _ctx_vectors()
    for case in g["cases"]:
        msg = wl.gen_chunk(g["seed"], case["id"], sum(case["pieces"])).tobytes()
        ctx = cio.Sha1() if engine == "library" else Sha1Ctx()
        state = (lambda: ctx.state) if engine == "library" else ctx.raw
        assert state().hex() == case["ctx_after_each"][0]
        pos = 0
        for k, ln in enumerate(case["pieces"]):
            ctx.update(msg[pos:pos + ln])
            pos += ln
            assert state().hex() == case["ctx_after_each"][k + 1], (case["id"], k)
        assert ctx.final().hex() == case["digest"]
        assert state().hex() == case["ctx_after_final"]
