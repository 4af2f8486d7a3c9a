#!/usr/bin/env python3
"""Golden SHA_CTX vectors from OpenSSL itself (tests/golden/sha1_ctx_vectors.json).

chunkio's cio_sha1 carries OpenSSL's SHA_CTX (include/chunkio/cio_sha1.h:25-27)
and cio_sha1_hash exports it before SHA1_Final (src/cio_sha1.c:52-54).  This
script records, for deterministic messages (chunkio_amd.workloads.gen_chunk:
the same splitmix64 bytes the GPU's fill kernel writes) cut at fixed split
points, the 96 context bytes libcrypto's SHA1_Init / SHA1_Update leave after
every piece, the context after SHA1_Final and the digest.  The tests check the
library's host SHA-1, the GPU batch calls and oracle/sha1_ctx.py against these
bytes, so the parity holds on a box where libcrypto cannot be loaded.

    python tests/golden/make_sha1_ctx.py      # rewrites the JSON (needs libcrypto)
"""
import ctypes
import ctypes.util
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from chunkio_amd import workloads as wl  # noqa: E402

SEED = 0x5A1C7
# (chunk id, pieces): padding edges (55/56/63/64/65), empty pieces, a piece
# that completes a pending block, long pieces
CASES = [(0, [3]), (1, [55]), (2, [56]), (3, [63]), (4, [64]), (5, [65]), (6, [0, 0, 1]),
         (7, [1, 63, 64, 0, 119]), (8, [60, 4, 60, 4]), (9, [1000, 3000, 5]),
         (10, [4096, 1, 4095]), (11, [65536 + 17]), (12, [10, 100, 1000, 10000]),
         (13, [409600 - 7, 7]), (14, [127, 128, 129, 130])]


def main():
    name = ctypes.util.find_library("crypto")
    if not name:
        sys.exit("libcrypto not found")
    c = ctypes.CDLL(name)
    c.SHA1_Update.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    out = {"generator": "tests/golden/make_sha1_ctx.py", "openssl": c.OpenSSL_version_num(),
           "message": "chunkio_amd.workloads.gen_chunk(seed, id, sum(pieces))", "seed": SEED, "cases": []}
    for cid, pieces in CASES:
        msg = wl.gen_chunk(SEED, cid, sum(pieces)).tobytes()
        ctx = ctypes.create_string_buffer(96)
        c.SHA1_Init(ctx)
        after, pos = [ctx.raw.hex()], 0
        for ln in pieces:
            c.SHA1_Update(ctx, msg[pos:pos + ln], ln)
            pos += ln
            after.append(ctx.raw.hex())
        md = ctypes.create_string_buffer(20)
        c.SHA1_Final(md, ctx)
        assert md.raw == hashlib.sha1(msg).digest()
        out["cases"].append({"id": cid, "pieces": pieces, "ctx_after_each": after,
                             "ctx_after_final": ctx.raw.hex(), "digest": md.raw.hex()})
    with open(os.path.join(HERE, "sha1_ctx_vectors.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"{len(out['cases'])} cases")


if __name__ == "__main__":
    main()
