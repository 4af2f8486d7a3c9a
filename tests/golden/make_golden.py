"""Generate tests/golden/crc32_vectors.json.

Every value is computed with the reference's own deps/crc32/crc32.c
(oracle/_ref/libcrc32_ref.so, built from /root/reference by oracle/Makefile)
AND cross-checked with Python's zlib.crc32; the script refuses to write a
vector on which the two disagree.  Inputs are either literal bytes, the
reference's own fixture tests/data/400kb.txt (copied here as data), or the
deterministic splitmix64 generator of chunkio_amd/workloads.py (parameters
stored, not bytes).

Run from the repo root:  python tests/golden/make_golden.py [--jobs-only]
"""
import hashlib
import json
import multiprocessing
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from chunkio_amd import workloads as wl  # noqa: E402
from oracle import pyoracle  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
D400 = open(os.path.join(HERE, "400kb.txt"), "rb").read()
INIT = 0xFFFFFFFF


def ref_raw(seed, data):
    r = pyoracle.crc_update_ref(seed, data)
    if seed == INIT:
        z = zlib.crc32(bytes(data)) ^ 0xFFFFFFFF
        assert r == z, (hex(r), hex(z))
    return r


def _cfg4_raw(i):
    return ref_raw(INIT, wl.gen_chunk(wl.CFG4_SEED, i, wl.CFG4_LEN).tobytes())


_L3 = None


def _cfg3_raw(i):
    global _L3
    if _L3 is None:
        _L3 = wl.cfg3_lens()
    return ref_raw(INIT, wl.gen_chunk(wl.CFG3_SEED, i, int(_L3[i])).tobytes())


def _cfg5_digest(i):
    return hashlib.sha1(wl.gen_chunk(wl.CFG2_SEED, i, wl.CFG2_LEN).tobytes()).digest()


# Weak-scaled jobs at N GPUs (bench.py --gpus N): chunk ids 0 .. N*n-1 of the
# config, rank r owning ids r, r+N, ...  Chunk i's bytes and length depend on i
# only, so the N-GPU job is the first N*n chunks of the 8-GPU one and one pass
# over 8*n chunks pins every N = 1..8 by prefix digests.
MAX_GPUS = 8
_L3J = None


def _cfg2_raw(i):
    return ref_raw(INIT, wl.gen_chunk(wl.CFG2_SEED, i, wl.CFG2_LEN).tobytes())


def _cfg4k_raw(i):
    return ref_raw(INIT, wl.gen_chunk(wl.CFG4K_SEED, i, wl.CFG4K_LEN).tobytes())


def _cfg3_raw_job(i):
    global _L3J
    if _L3J is None:
        _L3J = wl.cfg3_lens(MAX_GPUS * wl.CFG3_N)
    return ref_raw(INIT, wl.gen_chunk(wl.CFG3_SEED, i, int(_L3J[i])).tobytes())


def weak_jobs():
    """SHA-256 of the raw CRCs (SHA-1 digests for sha1) of the N-GPU job, in
    job order, for N = 1..8."""
    out = {"note": "bench.py weak configs at N GPUs: ids 0..N*n-1 (rank r owns r, r+N, ...); "
                   "sha256 of the job's raw CRCs as little-endian u32 (sha1: of the concatenated "
                   "20-byte digests); ids past n use the same generator (chunkio_amd/workloads.py)"}
    jobs = (("cfg2", _cfg2_raw, wl.CFG2_N, 32), ("cfg4k", _cfg4k_raw, wl.CFG4K_N, 4096),
            ("cfg3", _cfg3_raw_job, wl.CFG3_N, 256))
    for name, fn, n, cs in jobs:
        with multiprocessing.Pool(7) as pool:
            raw = np.asarray(pool.map(fn, range(MAX_GPUS * n), chunksize=cs), np.uint32)
        out[name] = {str(g): hashlib.sha256(raw[: g * n].astype("<u4").tobytes()).hexdigest()
                     for g in range(1, MAX_GPUS + 1)}
        print(name, "done", flush=True)
    with multiprocessing.Pool(7) as pool:
        dg = pool.map(_cfg5_digest, range(MAX_GPUS * wl.CFG2_N), chunksize=32)
    out["sha1"] = {str(g): hashlib.sha256(b"".join(dg[: g * wl.CFG2_N])).hexdigest()
                   for g in range(1, MAX_GPUS + 1)}
    return out


def main():
    if pyoracle.ref() is None:
        sys.exit("oracle/_ref/libcrc32_ref.so missing: run `make -C oracle` with /root/reference present")
    path = os.path.join(HERE, "crc32_vectors.json")
    if "--jobs-only" in sys.argv:
        # refresh only the weak-job digests of an existing fixture
        with open(path) as f:
            out = json.load(f)
        out["weak_jobs"] = weak_jobs()
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        print("wrote", path)
        return
    out = {"generator": "tests/golden/make_golden.py",
           "crc_model": "CRC-32/IEEE reflected 0xEDB88320; values are RAW crc_update states "
                        "(seed in, un-finalized out); finalized = raw ^ 0xffffffff"}

    kats = [
        ("check_123456789", b"123456789"),
        ("empty", b""),
        ("meta_len_field_fs.c:201", b"\x00\x00"),
        ("zero2_400kb_fs.c:209", b"\x00\x00" + D400),
        ("400kb", D400),
        ("zero2_5x400kb_cio_perf_file", b"\x00\x00" + D400 * 5),
        ("meta4_123456789", b"\x00\x04meta123456789"),
    ]
    out["kats"] = []
    for name, data in kats:
        raw = ref_raw(INIT, data)
        spec = {"name": name, "raw": raw, "crc32": raw ^ 0xFFFFFFFF, "len": len(data)}
        if len(data) <= 64:
            spec["hex"] = data.hex()
        else:
            spec["bytes"] = name  # reconstructed in the tests from 400kb.txt
        out["kats"].append(spec)
    # The reference's own expectations (tests/fs.c:201-214) as finalized CRCs.
    out["reference_expect"] = {"zero2": 0x41D912FF, "zero2_400kb": 0x103CFA67}

    # Random buffers for every length 0..4096 (seed 0x5EED, chunk index = length).
    rs = 0x5EED
    out["random_by_len"] = {"seed": rs, "max_len": 4096,
                            "raw": [ref_raw(INIT, wl.gen_chunk(rs, n, n).tobytes()) for n in range(4097)]}
    # Non-default raw seeds (continuation states), fixed data.
    seeds = [0, 0xBE26ED00, 0x12345678, 0xFFFFFFFF, 0x80000000, 0x00000001]
    lens = [1, 3, 4, 5, 15, 16, 17, 63, 64, 65, 4095, 4096, 4097, 10000, 409600]
    cont = []
    for s in seeds:
        for n in lens:
            data = wl.gen_chunk(0xABCD, n, n).tobytes()
            cont.append({"seed": s, "len": n, "raw": ref_raw(s, data)})
    out["seeded"] = {"data_seed": 0xABCD, "vectors": cont}

    # Config 2 batch: per-chunk raw CRCs of the first 32 chunks + digest of all.
    c2 = [ref_raw(INIT, wl.gen_chunk(wl.CFG2_SEED, i, wl.CFG2_LEN).tobytes()) for i in range(wl.CFG2_N)]
    out["cfg2"] = {"seed": wl.CFG2_SEED, "n": wl.CFG2_N, "len": wl.CFG2_LEN, "first32": c2[:32],
                   "sha256_of_raw_le": hashlib.sha256(np.asarray(c2, np.uint32).tobytes()).hexdigest()}
    # Config 3: geometry digest, raw CRCs of 48 spread chunks, and a digest of
    # all 65,536 raw CRCs (39.7 GB through the reference crc32.c and zlib, 6
    # processes), so the full batch is pinned whole, not by samples.
    l3 = wl.cfg3_lens()
    idx3 = [int(x) for x in np.linspace(0, wl.CFG3_N - 1, 48).astype(int)]
    with multiprocessing.Pool(6) as pool:
        c3 = pool.map(_cfg3_raw, range(wl.CFG3_N), chunksize=256)
    out["cfg3"] = {"seed": wl.CFG3_SEED, "n": wl.CFG3_N, "total_bytes": int(l3.sum()),
                   "min_len": int(l3.min()), "max_len": int(l3.max()),
                   "lens_sha256": hashlib.sha256(l3.astype("<u8").tobytes()).hexdigest(),
                   "sample_idx": idx3,
                   "sample_raw": [c3[i] for i in idx3],
                   "sha256_of_raw_le": hashlib.sha256(np.asarray(c3, np.uint32).tobytes()).hexdigest()}
    # Config 4: raw CRCs of 8 chunks (one per GPU shard at G=8), and a digest of
    # all 8192 (34.4 GB through the reference crc32.c and zlib, 6 processes),
    # so the sharded full-size job can be checked whole.
    with multiprocessing.Pool(6) as pool:
        c4 = pool.map(_cfg4_raw, range(wl.CFG4_N), chunksize=64)
    out["cfg4"] = {"seed": wl.CFG4_SEED, "n": wl.CFG4_N, "len": wl.CFG4_LEN,
                   "sample_idx": list(range(8)),
                   "sample_raw": c4[:8],
                   "sha256_of_raw_le": hashlib.sha256(np.asarray(c4, np.uint32).tobytes()).hexdigest()}
    # SHA-1 (config 5): hashlib (OpenSSL) -- the reference's <sha1/sha1.h> is not vendored.
    # All 1,024 cfg2-batch digests are pinned by the SHA-256 of their concatenation.
    with multiprocessing.Pool(6) as pool:
        c5 = pool.map(_cfg5_digest, range(wl.CFG2_N), chunksize=32)
    out["sha1"] = {"oracle": "hashlib.sha1 (OpenSSL); FIPS 180-4 KATs",
                   "kats": [{"hex": b"abc".hex(), "digest": hashlib.sha1(b"abc").hexdigest()},
                            {"hex": "", "digest": hashlib.sha1(b"").hexdigest()},
                            {"hex": b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq".hex(),
                             "digest": "84983e441c3bd26ebaae4aa1f95129e5e54670f1"}],
                   "cfg2_first8": [d.hex() for d in c5[:8]],
                   "cfg5_n": wl.CFG2_N,
                   "cfg5_sha256_of_digests": hashlib.sha256(b"".join(c5)).hexdigest(),
                   "400kb": hashlib.sha1(D400).hexdigest()}
    out["weak_jobs"] = weak_jobs()
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", os.path.join(HERE, "crc32_vectors.json"))


if __name__ == "__main__":
    main()
