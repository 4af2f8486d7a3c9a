"""Chunk files written, damaged and loaded by the REFERENCE chunkio
(tests/golden/chunks/, made by gen_ref_chunks.c through make_ref_chunks.py
against the reference built in /tmp by its own CMake).

  * replay: the same operations through this repo's chunk layer
    (cioa_chunk.c; immediate and deferred CRC) plus the same damage give
    byte-identical files (src/cio_file.c:994-1073 write, :1147-1250 sync,
    :130-146 adjust_layout, src/cio_chunk.c:184-209 write_at);
  * verify: cio_verify_paths gives, per file, the reference loader's verdict
    (src/cio_scan.c:102-105 -> cio_file_format_check, src/cio_file.c:187-294):
    status, error code, and for a loaded chunk its crc_cur; with
    CIOA_VERIFY_WRITEBACK the files end as the reference's load left them
    (legacy length written back, cio_file_st.h:160-175);
  * scan: Context.scan of the whole stream reports the same chunks loaded.

Each runs on the host CRC route in the CPU suite and on the GPU route
(cio_crc32_set_cpu_max(0)) under -m gpu."""
import hashlib
import json
import os
import shutil

import numpy as np
import pytest

from chunkio_amd import chunkfile as cf

HERE = os.path.dirname(os.path.abspath(__file__))
GDIR = os.path.join(HERE, "golden", "chunks")
with open(os.path.join(GDIR, "manifest.json")) as _f:
    MANIFEST = json.load(_f)
CHUNKS = MANIFEST["chunks"]
NAMES = [c["name"] for c in CHUNKS]

ROUTES = [pytest.param("host", id="host"), pytest.param("gpu", marks=pytest.mark.gpu, id="gpu"),
          pytest.param("split", marks=pytest.mark.gpu, id="split")]


@pytest.fixture
def route(request):
    import chunkio_amd as cio
    if request.param == "gpu":
        request.getfixturevalue("cuda")
        cio.route(reset=True, cpu_max=0)
    elif request.param == "split":
        # every batch of two or more chunks shared: the first chunks on the
        # GPU (helper thread), the rest on the calling thread's host CRC
        request.getfixturevalue("cuda")
        cio.route(reset=True, cpu_max=1, threads=1, split="force")
    else:
        cio.route(reset=True, cpu_max=1 << 62, threads=1)
    yield request.param
    cio.route(reset=True)


def pattern(n, seed):
    i = np.arange(n, dtype=np.uint64)
    return (((i * 131 + seed * 7 + 17) % 251) + 1).astype(np.uint8).tobytes()


def sha(b):
    return hashlib.sha256(b).hexdigest()


def fixture_bytes(name):
    with open(os.path.join(GDIR, "files", name), "rb") as f:
        return f.read()


def apply_post(path, post):
    for p in post:
        if p["op"] == "patch":
            with open(path, "r+b") as f:
                f.seek(p["offset"])
                f.write(bytes.fromhex(p["hex"]))
        elif p["op"] == "xor":
            with open(path, "r+b") as f:
                f.seek(p["offset"])
                b = f.read(1)[0] ^ p["mask"]
                f.seek(p["offset"])
                f.write(bytes([b]))
        elif p["op"] == "truncate":
            os.truncate(path, p["size"])
        else:
            raise ValueError(p)


def replay(root, spec, deferred):
    """The scenario's calls on this repo's chunk layer, in a private context
    rooted at `root` with the scenario's context flags."""
    flags = spec["ctx_flags"] | (cf.CIOA_DEFERRED_CRC if deferred else 0)
    with cf.Context(root, flags) as ctx:
        st = ctx.stream(MANIFEST["stream"])
        c, err = st.open(spec["name"], cf.CIO_OPEN, spec["open_size"])
        assert c is not None, err
        for op in spec["ops"]:
            if op["op"] == "write":
                assert c.write(pattern(op["len"], op["seed"])) == 0
            elif op["op"] == "write_at":
                assert c.write_at(pattern(op["len"], op["seed"]), op["offset"]) == 0
            elif op["op"] == "meta_write":
                assert c.meta_write(op["meta"].encode()) == 0
            elif op["op"] == "sync":
                assert c.sync() == op["rc"]
            elif op["op"] == "close":
                c.close()
            else:
                raise ValueError(op)
    path = os.path.join(root, MANIFEST["stream"], spec["name"])
    apply_post(path, spec.get("post", []))
    return path


def test_fixture_integrity():
    """The committed files are the ones the reference wrote (size, SHA-256),
    and the manifest covers every case the verify path distinguishes."""
    assert len(CHUNKS) >= 6
    for s in CHUNKS:
        b = fixture_bytes(s["name"])
        assert len(b) == s["size"] and sha(b) == s["sha256"], s["name"]
    errs = {s["load"]["last_chunk_error"] for s in CHUNKS}
    assert errs >= {0, cf.CIO_ERR_BAD_CHECKSUM, cf.CIO_ERR_BAD_LAYOUT, cf.CIO_ERR_BAD_FILE_SIZE}
    by = {s["name"]: s for s in CHUNKS}
    # the empty chunk's header is tests/fs.c:201-206's 41 d9 12 ff
    assert fixture_bytes("c01_empty")[2:10] == bytes.fromhex("41d912ff00000000")
    assert by["c01_empty"]["load"]["crc_cur"] == 0xBE26ED00
    # a legacy file loads, and the load writes its inferred length back
    assert by["c07_legacy_exact"]["load"]["ok"]
    assert by["c07_legacy_exact"]["sha256_after_load"] != by["c07_legacy_exact"]["sha256"]


@pytest.mark.parametrize("deferred", [False, pytest.param(True, id="deferred")])
@pytest.mark.parametrize("route", ROUTES, indirect=True)
def test_replay_is_byte_identical(route, deferred, tmp_path):
    """Every scenario's operations through cioa_chunk.c (immediate per-write
    CRC, or deferred CRC computed in one routed batch at sync) write the
    reference's bytes exactly, including the damaged variants."""
    diffs = []
    for s in CHUNKS:
        path = replay(str(tmp_path / ("d" if deferred else "i")), s, deferred)
        with open(path, "rb") as f:
            got = f.read()
        want = fixture_bytes(s["name"])
        if got != want:
            first = next((i for i in range(min(len(got), len(want))) if got[i] != want[i]), None)
            diffs.append((s["name"], len(got), len(want), first))
    assert not diffs, diffs


def _copy_stream(tmp_path):
    d = tmp_path / "root" / MANIFEST["stream"]
    d.mkdir(parents=True)
    for n in NAMES:
        shutil.copyfile(os.path.join(GDIR, "files", n), d / n)
    return d


def _verdicts(st, er, cr, names, flags_of):
    out = {}
    for i, n in enumerate(names):
        out[n] = (int(st[i]), int(er[i]), int(cr[i]) if int(st[i]) == cf.CIO_OK and flags_of(n) else None)
    return out


def _expected(names):
    by = {s["name"]: s for s in CHUNKS}
    out = {}
    for n in names:
        ld = by[n]["load"]
        status = cf.CIO_OK if ld["ok"] else ld["err"]
        crc = ld["crc_cur"] if ld["ok"] and by[n]["load_flags"] & cf.CIO_CHECKSUM else None
        out[n] = (status, ld["last_chunk_error"], crc)
    return out


@pytest.mark.parametrize("route", ROUTES, indirect=True)
def test_verify_paths_matches_reference_loader(route, tmp_path):
    """cio_verify_paths over the reference's files: the reference loader's
    status / error / crc_cur per file, read-only (files unchanged) and with
    CIOA_VERIFY_WRITEBACK (files left as the reference's load left them)."""
    d = _copy_stream(tmp_path)
    by = {s["name"]: s for s in CHUNKS}
    expected = _expected(NAMES)
    for load_flags in sorted({s["load_flags"] for s in CHUNKS}):
        names = [n for n in NAMES if by[n]["load_flags"] == load_flags]
        paths = [str(d / n) for n in names]
        st, er, cr = cf.verify_paths(paths, flags=load_flags)
        got = _verdicts(st, er, cr, names, lambda n: by[n]["load_flags"] & cf.CIO_CHECKSUM)
        assert got == {n: expected[n] for n in names}
        for n in names:   # read-only: nothing written
            assert sha(open(d / n, "rb").read()) == by[n]["sha256"], n
        st, er, cr = cf.verify_paths(paths, flags=load_flags | cf.CIOA_VERIFY_WRITEBACK)
        got = _verdicts(st, er, cr, names, lambda n: by[n]["load_flags"] & cf.CIO_CHECKSUM)
        assert got == {n: expected[n] for n in names}
        for n in names:
            assert sha(open(d / n, "rb").read()) == by[n]["sha256_after_load"], n


@pytest.mark.parametrize("route", ROUTES, indirect=True)
def test_scan_loads_what_the_reference_loads(route, tmp_path):
    """Context.scan (cio_scan_stream_files: one verify batch) over the
    checksummed fixtures: exactly the files the reference loaded come up,
    with the reference's crc_cur and content size; the rest are refused."""
    d = _copy_stream(tmp_path)
    by = {s["name"]: s for s in CHUNKS}
    for n in NAMES:
        if not by[n]["load_flags"] & cf.CIO_CHECKSUM:
            os.unlink(d / n)
    with cf.Context(str(tmp_path / "root"), cf.CIO_CHECKSUM) as ctx:
        _, chunks = ctx.scan(MANIFEST["stream"])
        loaded = {c.name: (c.crc_cur, c.data_size) for c in chunks}
    want = {n: (by[n]["load"]["crc_cur"], by[n]["load"]["content_size"])
            for n in NAMES if by[n]["load_flags"] & cf.CIO_CHECKSUM and by[n]["load"]["ok"]}
    assert loaded == want
