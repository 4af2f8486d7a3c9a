"""GPU parity for the batched SHA-1 content hash (BASELINE config 5).

Oracle: hashlib.sha1 (OpenSSL) plus FIPS 180-4 known answers; the reference's
<sha1/sha1.h> (include/chunkio/cio_sha1.h:52) is third-party and not vendored,
so this path is pinned by the standard's vectors, not by reference fixtures.
"""
import hashlib

import numpy as np
import pytest

import chunkio_amd as cio
from chunkio_amd import workloads as wl

pytestmark = pytest.mark.gpu


def run(cuda, chunks, misalign=0):
    from test_gpu_crc import pack, to_dev
    buf, offs, lens = pack(chunks, misalign=[misalign] * len(chunks))
    return cio.sha1_batch_dev(to_dev(buf, cuda), offs, lens)


def test_fips_kats(cuda, golden):
    chunks = [bytes.fromhex(k["hex"]) for k in golden["sha1"]["kats"]]
    for mis in (0, 3):
        got = run(cuda, chunks, mis)
        assert [bytes(d).hex() for d in got] == [k["digest"] for k in golden["sha1"]["kats"]]


def test_padding_boundaries(cuda):
    rng = np.random.default_rng(21)
    lens = list(range(0, 200)) + [447, 448, 449, 511, 512, 513, 4095, 4096, 4097, 100003]
    chunks = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    for mis in (0, 1, 8):
        got = run(cuda, chunks, mis)
        for c, d in zip(chunks, got):
            assert bytes(d) == hashlib.sha1(c).digest(), len(c)


def test_cfg5_full_batch(cuda, golden, data400):
    """All 1,024 cfg5 digests, pinned by the SHA-256 of their concatenation
    (hashlib, tests/golden/make_golden.py)."""
    import torch
    lens = wl.cfg2_lens()
    offs = wl.packed_offsets(lens)
    dev = torch.empty(wl.batch_bytes(offs, lens), dtype=torch.uint8, device=cuda)
    cio.fill_synthetic(dev, offs, lens, wl.CFG2_SEED)
    got = cio.sha1_batch_dev(dev, offs, lens)
    assert [bytes(d).hex() for d in got[:8]] == golden["sha1"]["cfg2_first8"]
    assert hashlib.sha256(got.tobytes()).hexdigest() == golden["sha1"]["cfg5_sha256_of_digests"]
    got400 = run(cuda, [data400])
    assert bytes(got400[0]).hex() == golden["sha1"]["400kb"]


def test_async_device_descriptors(cuda, golden):
    """cio_sha1_batch_dev_async (device-resident offsets/lengths, no sync) gives
    the digests of the synchronous entry on the full cfg5 batch, repeated on one
    stream, and on ragged lengths whose lanes end at different blocks."""
    import torch
    lens = wl.cfg2_lens()
    offs = wl.packed_offsets(lens, align=16)
    dev = torch.empty(wl.batch_bytes(offs, lens) + 64, dtype=torch.uint8, device=cuda)
    cio.fill_synthetic(dev, offs, lens, wl.CFG2_SEED)
    want = cio.sha1_batch_dev(dev, offs, lens)
    assert [bytes(d).hex() for d in want[:8]] == golden["sha1"]["cfg2_first8"]
    assert hashlib.sha256(want.tobytes()).hexdigest() == golden["sha1"]["cfg5_sha256_of_digests"]
    d_offs = torch.from_numpy(offs.astype(np.int64)).to(cuda)
    d_lens = torch.from_numpy(lens.astype(np.int64)).to(cuda)
    out = torch.zeros(len(lens) * 20, dtype=torch.uint8, device=cuda)
    for _ in range(3):
        cio.sha1_batch_dev_async(dev, d_offs, d_lens, out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().reshape(-1, 20), want)
    assert hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest() == golden["sha1"]["cfg5_sha256_of_digests"]

    rng = np.random.default_rng(22)
    rl = rng.integers(0, 20000, 200).astype(np.uint64)
    ro = wl.packed_offsets(rl)
    rdev = torch.empty(wl.batch_bytes(ro, rl) + 64, dtype=torch.uint8, device=cuda)
    cio.fill_synthetic(rdev, ro, rl, 0x5A1)
    rout = torch.zeros(len(rl) * 20, dtype=torch.uint8, device=cuda)
    cio.sha1_batch_dev_async(rdev, torch.from_numpy(ro.astype(np.int64)).to(cuda),
                             torch.from_numpy(rl.astype(np.int64)).to(cuda), rout)
    got = rout.cpu().numpy().reshape(-1, 20)
    host = rdev.cpu().numpy()
    for i in range(len(rl)):
        assert bytes(got[i]) == hashlib.sha1(host[int(ro[i]):int(ro[i] + rl[i])].tobytes()).digest(), i


def test_many_workgroups_ragged_and_misaligned(cuda):
    """20,011 chunks (626 workgroups of 32 chunks, more than one per CU) with
    lengths 0..3000 at arbitrary byte offsets: lanes of one wave end at
    different blocks and most take the byte-wise message path."""
    import torch
    rng = np.random.default_rng(23)
    n = 20011
    lens = rng.integers(0, 3001, n).astype(np.uint64)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1] + rng.integers(0, 16, n - 1).astype(np.uint64))
    total = int(offs[-1] + lens[-1]) + 64
    host = rng.integers(0, 256, total, dtype=np.uint8)
    dev = torch.from_numpy(host).to(cuda)
    got = cio.sha1_batch_dev(dev, offs, lens)
    for i in range(n):
        o, ln = int(offs[i]), int(lens[i])
        assert bytes(got[i]) == hashlib.sha1(host[o:o + ln].tobytes()).digest(), i


def test_bit_length_high_word(cuda):
    """A chunk of 512 MiB + 77 bytes: the 64-bit message bit length in the
    padding has a non-zero high word (FIPS 180-4 5.1.1), one-shot and through
    SHA1_Update (two pieces) + SHA1_Final.  One serial chain: ~7 s each."""
    import torch
    n = (512 << 20) + 77
    gen = torch.Generator(device=cuda)
    gen.manual_seed(0x5A1B)
    dev = torch.randint(0, 256, (n + 64,), dtype=torch.uint8, device=cuda, generator=gen)
    host = dev.cpu().numpy()
    want = hashlib.sha1(host[3:3 + n].tobytes()).digest()
    got = cio.sha1_batch_dev(dev, np.array([3], np.uint64), np.array([n], np.uint64))
    assert bytes(got[0]) == want
    states = cio.sha1_states_init(1, cuda)
    cut = (300 << 20) + 5
    cio.sha1_update_batch_dev(dev, _dev_i64([3], cuda), _dev_i64([cut], cuda), states)
    cio.sha1_update_batch_dev(dev, _dev_i64([3 + cut], cuda), _dev_i64([n - cut], cuda), states)
    assert bytes(cio.sha1_final_batch_dev(states)[0]) == want


@pytest.mark.parametrize("update", [False, True])
def test_select_free_groups(cuda, update):
    """The round wave runs the groups every chunk of its workgroup has in full
    without per-lane selects, then the rest with them.  Workgroups (32 chunks)
    of equal lengths whose block count is a multiple of the 4-block group, one
    more, three more; one with a single empty chunk (no select-free group); one
    with a single long chunk among short ones; a partial last workgroup.  Both
    the one-shot digest and SHA1_Update + SHA1_Final."""
    import torch
    rng = np.random.default_rng(24)
    groups = [
        [64 * 40 - 9] * 32,                       # 40 blocks with padding: 10 whole groups
        [64 * 41 - 9] * 32,                       # 41 blocks
        [64 * 43 - 9] * 32,                       # 43 blocks
        [0] + [64 * 40] * 31,                     # one empty chunk
        [5000] + [100] * 31,                      # one long chunk
        [64 * 12 + 5] * 7,                        # partial workgroup
    ]
    lens = np.array([x for g in groups for x in g], np.uint64)
    offs = wl.packed_offsets(lens, align=16)
    total = int(offs[-1] + lens[-1]) + 64
    host = rng.integers(0, 256, total, dtype=np.uint8)
    dev = torch.from_numpy(host).to(cuda)
    if update:
        states = cio.sha1_states_init(len(lens), cuda)
        cio.sha1_update_batch_dev(dev, _dev_i64(offs, cuda), _dev_i64(lens, cuda), states)
        got = cio.sha1_final_batch_dev(states)
    else:
        got = cio.sha1_batch_dev(dev, offs, lens)
    for i in range(len(lens)):
        o, ln = int(offs[i]), int(lens[i])
        assert bytes(got[i]) == hashlib.sha1(host[o:o + ln].tobytes()).digest(), i


def test_block_count_boundaries(cuda):
    """Block counts 1 .. 97 around multiples of 4 and 16 (the kernel's 4-block
    hand-over groups), cycled so that the chunks of one workgroup end in
    different groups, aligned and misaligned, 1100 chunks (more workgroups
    than CUs at 8 chunks per workgroup)."""
    import torch
    rng = np.random.default_rng(25)
    nblks = [1, 15, 16, 17, 31, 32, 33, 47, 48, 49, 63, 64, 65, 95, 96, 97]
    # nblk = full + 1 when the tail is < 56 bytes (a 10-byte tail: one padding block)
    base_lens = [64 * (b - 1) + 10 for b in nblks] + [64 * 47 + 60]   # the last: 49 blocks (2 padding)
    lens = np.array([base_lens[(i * 7) % len(base_lens)] for i in range(1100)], np.uint64)
    for align in (16, 1):
        offs = wl.packed_offsets(lens, align=align, start=0 if align == 16 else 3)
        total = int(offs[-1] + lens[-1]) + 64
        host = rng.integers(0, 256, total, dtype=np.uint8)
        dev = torch.from_numpy(host).to(cuda)
        got = cio.sha1_batch_dev(dev, offs, lens)
        for i in range(len(lens)):
            o, ln = int(offs[i]), int(lens[i])
            assert bytes(got[i]) == hashlib.sha1(host[o:o + ln].tobytes()).digest(), (align, i, ln)


def test_concurrent_streams(cuda):
    """Batches on four streams from four threads, three launches each: every
    batch gets its own digests (the A/B one-chunk-per-wave kernel's per-device
    ring is ordered across streams through an event)."""
    import threading

    import torch
    rng = np.random.default_rng(26)
    jobs = []
    for t in range(4):
        lens = rng.integers(0, 40000, 300 + 50 * t).astype(np.uint64)
        offs = wl.packed_offsets(lens, align=16)
        host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
        jobs.append((torch.from_numpy(host).to(cuda), offs, lens, host))
    torch.cuda.synchronize()
    results = [None] * len(jobs)

    def work(t):
        dev, offs, lens, _ = jobs[t]
        s = torch.cuda.Stream(device=cuda)
        with torch.cuda.stream(s):
            for _ in range(3):
                results[t] = cio.sha1_batch_dev(dev, offs, lens, stream=s)

    threads = [threading.Thread(target=work, args=(t,)) for t in range(len(jobs))]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    for (dev, offs, lens, host), got in zip(jobs, results):
        for i in range(len(lens)):
            o, ln = int(offs[i]), int(lens[i])
            assert bytes(got[i]) == hashlib.sha1(host[o:o + ln].tobytes()).digest(), i


# ---- continuation: SHA1_Init / SHA1_Update / SHA1_Final per chunk ---------
# (cio_sha1_update_batch_dev / cio_sha1_final_batch_dev; the reference's
# cio_sha1_init/update/final, src/cio_sha1.c:26-39, and the pre-Final state
# export of cio_sha1_hash, :41-57)

def _dev_i64(a, cuda):
    import torch
    return torch.from_numpy(np.asarray(a, dtype=np.int64)).to(cuda)


def test_continuation_random_splits(cuda):
    """Three updates per chunk at random split points (any byte, not only
    64-byte multiples, empty pieces included), the byte stream contiguous in
    memory at random 16-byte-aligned and unaligned bases: after every update
    the final digest equals hashlib over the prefix, and the exported state
    holds the prefix's byte count and pending tail."""
    import torch
    rng = np.random.default_rng(71)
    n = 300
    lens = rng.integers(0, 20000, n).astype(np.uint64)
    lens[:8] = [0, 1, 63, 64, 65, 119, 128, 4096]
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1] + rng.integers(0, 40, n - 1).astype(np.uint64))
    host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    dev = torch.from_numpy(host).to(cuda)
    cuts = np.sort(np.stack([rng.integers(0, lens.astype(np.int64) + 1) for _ in range(2)], axis=1), axis=1)
    cuts[:40:4, 0] = (cuts[:40:4, 0] // 64) * 64          # some block-aligned splits
    bounds = np.concatenate([np.zeros((n, 1), np.int64), cuts, lens.astype(np.int64)[:, None]], axis=1)
    states = cio.sha1_states_init(n, cuda)
    for stage in range(3):
        a, b = bounds[:, stage], bounds[:, stage + 1]
        cio.sha1_update_batch_dev(dev, _dev_i64(offs.astype(np.int64) + a, cuda), _dev_i64(b - a, cuda), states)
        got = cio.sha1_final_batch_dev(states)
        view = cio.sha1_states_view(states)
        for i in range(n):
            pre = host[int(offs[i]):int(offs[i]) + int(b[i])].tobytes()
            assert bytes(got[i]) == hashlib.sha1(pre).digest(), (stage, i)
            assert int(view["bits"][i]) == 8 * len(pre) and int(view["num"][i]) == len(pre) % 64, (stage, i)
            k = len(pre) % 64
            assert view["data"][i, :k].tobytes() == pre[len(pre) - k:], (stage, i)
            assert not view["data"][i, k:].any(), (stage, i)
            # the whole context is the host SHA-1's (pinned to OpenSSL's SHA_CTX
            # bytes by tests/test_sha1_host.py) after the same updates
            ref = cio.Sha1()
            for s0 in range(stage + 1):
                ref.update(host[int(offs[i]) + int(bounds[i, s0]):int(offs[i]) + int(bounds[i, s0 + 1])])
            assert view["raw"][i].tobytes() == ref.state, (stage, i)
    # the full-message digests also equal the one-shot kernel's
    assert np.array_equal(cio.sha1_final_batch_dev(states), cio.sha1_batch_dev(dev, offs, lens))


def test_continuation_across_buffers_and_final_keeps_state(cuda):
    """A from one buffer, B from another at an unrelated (misaligned) address:
    the continued context is only the 96-byte state.  Final leaves the state
    untouched, so hashing continues after a digest was taken."""
    import torch
    rng = np.random.default_rng(72)
    n = 130
    la = rng.integers(0, 3000, n)
    lb = rng.integers(0, 3000, n)
    A = [rng.integers(0, 256, int(x), dtype=np.uint8).tobytes() for x in la]
    B = [rng.integers(0, 256, int(x), dtype=np.uint8).tobytes() for x in lb]
    from test_gpu_crc import pack, to_dev
    bufa, oa, _ = pack(A, misalign=[int(x) for x in rng.integers(0, 16, n)])
    bufb, ob, _ = pack(B, misalign=[int(x) for x in rng.integers(0, 16, n)])
    da, db = to_dev(bufa, cuda), to_dev(bufb, cuda)
    states = cio.sha1_states_init(n, cuda)
    cio.sha1_update_batch_dev(da, _dev_i64(oa, cuda), _dev_i64(la, cuda), states)
    before = states.clone()
    got_a = cio.sha1_final_batch_dev(states)
    assert torch.equal(states, before)
    assert [bytes(d) for d in got_a] == [hashlib.sha1(x).digest() for x in A]
    cio.sha1_update_batch_dev(db, _dev_i64(ob, cuda), _dev_i64(lb, cuda), states)
    cio.sha1_update_batch_dev(db, _dev_i64(ob, cuda), _dev_i64(np.zeros(n), cuda), states)   # empty updates
    got = cio.sha1_final_batch_dev(states)
    assert [bytes(d) for d in got] == [hashlib.sha1(x + y).digest() for x, y in zip(A, B)]


def test_continuation_appends_cfg5_shape(cuda, golden):
    """The cfg5 batch hashed as a chunk grows in place: five 81,920-byte
    appends per 409,600-byte chunk (block-aligned stream, the fast path
    after block 0), then one 7-byte append per chunk and its digest."""
    import torch
    lens = wl.cfg2_lens()
    offs = wl.packed_offsets(lens, align=16)
    dev = torch.empty(wl.batch_bytes(offs, lens) + 64, dtype=torch.uint8, device=cuda)
    cio.fill_synthetic(dev, offs, lens, wl.CFG2_SEED)
    n = len(lens)
    states = cio.sha1_states_init(n, cuda)
    step = 81920
    for k in range(5):
        cio.sha1_update_batch_dev(dev, _dev_i64(offs.astype(np.int64) + k * step, cuda),
                                  _dev_i64(np.full(n, step), cuda), states)
    got = cio.sha1_final_batch_dev(states)
    assert [bytes(d).hex() for d in got[:8]] == golden["sha1"]["cfg2_first8"]
    assert hashlib.sha256(got.tobytes()).hexdigest() == golden["sha1"]["cfg5_sha256_of_digests"]
    assert np.array_equal(got, cio.sha1_batch_dev(dev, offs, lens))
    tail = torch.arange(7, dtype=torch.uint8, device=cuda) + 1
    cio.sha1_update_batch_dev(tail, _dev_i64(np.zeros(n), cuda), _dev_i64(np.full(n, 7), cuda), states)
    got7 = cio.sha1_final_batch_dev(states)
    host = dev.cpu().numpy()
    for i in (0, 511, n - 1):
        msg = host[int(offs[i]):int(offs[i] + lens[i])].tobytes() + bytes(range(1, 8))
        assert bytes(got7[i]) == hashlib.sha1(msg).digest(), i


# ---- SHA_CTX parity with OpenSSL: contexts cross between OpenSSL and the GPU --

def _openssl():
    import ctypes
    import ctypes.util
    name = ctypes.util.find_library("crypto")
    if not name:
        pytest.skip("OpenSSL libcrypto is not installed on this box")
    c = ctypes.CDLL(name)
    if not all(hasattr(c, f) for f in ("SHA1_Init", "SHA1_Update", "SHA1_Final")):
        pytest.skip("libcrypto lacks the SHA1_* API")
    c.SHA1_Init.argtypes = [ctypes.c_void_p]
    c.SHA1_Update.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    c.SHA1_Final.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    return c


def _ossl_ctx(c, state=None, data=b""):
    import ctypes
    buf = ctypes.create_string_buffer(96)
    if state is None:
        c.SHA1_Init(buf)
    else:
        ctypes.memmove(buf, bytes(state), 96)
    if data:
        c.SHA1_Update(buf, data, len(data))
    return buf


def _ossl_final(c, buf):
    import ctypes
    md = ctypes.create_string_buffer(20)
    c.SHA1_Final(md, buf)
    return md.raw


def test_openssl_contexts_continue_on_the_gpu_and_back(cuda):
    """Both directions, 257 chunks at random split points (padding edges
    included), data at misaligned device offsets:
      1. OpenSSL hashes a prefix; its 96 SHA_CTX bytes go to the device as is;
         cio_sha1_update_batch_dev adds the middle; the device context bytes
         equal OpenSSL's after prefix + middle;
      2. those device bytes go back to OpenSSL, which adds the suffix and
         finishes: the digest is the whole message's; the GPU's own final over
         the same context (cio_sha1_final_batch_dev) agrees at the middle."""
    import torch
    c = _openssl()
    rng = np.random.default_rng(81)
    n = 257
    edges = [0, 1, 55, 56, 57, 63, 64, 65, 119, 120, 128]
    pre_l = np.array([edges[i % len(edges)] if i < 60 else int(rng.integers(0, 5000)) for i in range(n)])
    mid_l = np.array([edges[(i * 3) % len(edges)] if i < 60 else int(rng.integers(0, 9000)) for i in range(n)])
    suf_l = rng.integers(0, 700, n)
    msgs = [rng.integers(0, 256, int(a + b + s), dtype=np.uint8).tobytes() for a, b, s in zip(pre_l, mid_l, suf_l)]
    from test_gpu_crc import pack, to_dev
    mids = [m[int(a):int(a + b)] for m, a, b in zip(msgs, pre_l, mid_l)]
    buf, offs, _ = pack(mids, misalign=[int(x) for x in rng.integers(0, 16, n)])
    dev = to_dev(buf, cuda)
    ctxs = [_ossl_ctx(c, data=m[:int(a)]) for m, a in zip(msgs, pre_l)]
    states = torch.from_numpy(np.frombuffer(b"".join(x.raw for x in ctxs), np.uint8).copy()).to(cuda)
    cio.sha1_update_batch_dev(dev, _dev_i64(offs, cuda), _dev_i64(mid_l, cuda), states)
    dig_mid = cio.sha1_final_batch_dev(states)
    raw = cio.sha1_states_view(states)["raw"]
    for i in range(n):
        upto = msgs[i][:int(pre_l[i] + mid_l[i])]
        want = _ossl_ctx(c, data=upto).raw
        assert raw[i].tobytes() == want, i
        assert bytes(dig_mid[i]) == hashlib.sha1(upto).digest(), i
        back = _ossl_ctx(c, state=raw[i].tobytes(), data=msgs[i][int(pre_l[i] + mid_l[i]):])
        assert _ossl_final(c, back) == hashlib.sha1(msgs[i]).digest(), i


def test_gpu_contexts_match_openssl_on_the_cfg5_batch(cuda):
    """The cfg5 batch (1024 x 409,600 B) hashed on the GPU as 409,593 + 7
    bytes per chunk: every one of the 1024 device contexts after the first
    update equals OpenSSL's SHA_CTX after the same bytes, and OpenSSL
    finishes each of them to the full chunk's digest."""
    import torch
    c = _openssl()
    lens = wl.cfg2_lens()
    offs = wl.packed_offsets(lens, align=16)
    dev = torch.empty(wl.batch_bytes(offs, lens) + 64, dtype=torch.uint8, device=cuda)
    cio.fill_synthetic(dev, offs, lens, wl.CFG2_SEED)
    n = len(lens)
    cut = 409593
    states = cio.sha1_states_init(n, cuda)
    cio.sha1_update_batch_dev(dev, _dev_i64(offs, cuda), _dev_i64(np.full(n, cut), cuda), states)
    raw = cio.sha1_states_view(states)["raw"]
    host = dev.cpu().numpy()
    for i in range(n):
        chunk = host[int(offs[i]):int(offs[i] + lens[i])].tobytes()
        assert raw[i].tobytes() == _ossl_ctx(c, data=chunk[:cut]).raw, i
        fin = _ossl_ctx(c, state=raw[i].tobytes(), data=chunk[cut:])
        assert _ossl_final(c, fin) == hashlib.sha1(chunk).digest(), i


def test_openssl_context_near_2_32_bits_continues_on_the_gpu(cuda):
    """A context OpenSSL built from 512 MiB - 3 bytes (Nl just below 2^32)
    continued on the GPU by 11 bytes: Nl wraps and Nh carries exactly as
    OpenSSL's own SHA1_Update does, and the digest is the whole message's."""
    import torch
    c = _openssl()
    rng = np.random.default_rng(84)
    block = rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes()
    ref = _ossl_ctx(c)
    h = hashlib.sha1()
    for _ in range(511):
        c.SHA1_Update(ref, block, len(block))
        h.update(block)
    tail = block[:(1 << 20) - 3]
    c.SHA1_Update(ref, tail, len(tail))
    h.update(tail)
    assert int.from_bytes(ref.raw[24:28], "little") == 0
    more = bytes(range(11))
    states = torch.from_numpy(np.frombuffer(ref.raw, np.uint8).copy()).to(cuda)
    dev = torch.from_numpy(np.frombuffer(more, np.uint8).copy()).to(cuda)
    cio.sha1_update_batch_dev(dev, _dev_i64([0], cuda), _dev_i64([len(more)], cuda), states)
    c.SHA1_Update(ref, more, len(more))
    h.update(more)
    raw = cio.sha1_states_view(states)["raw"][0].tobytes()
    assert raw == ref.raw and int.from_bytes(raw[24:28], "little") == 1
    assert bytes(cio.sha1_final_batch_dev(states)[0]) == h.digest()


def test_device_contexts_equal_the_context_oracle(cuda):
    """Without OpenSSL in the loop: the device contexts after random splits
    equal oracle/sha1_ctx.py's (pure-Python SHA_CTX restatement, pinned to
    libcrypto by tests/test_sha1_host.py), and an oracle-made context
    continued on the GPU finishes to hashlib's digest."""
    import torch
    from oracle.sha1_ctx import Sha1Ctx
    rng = np.random.default_rng(85)
    n = 96
    lens = rng.integers(0, 3000, n).astype(np.uint64)
    lens[:6] = [0, 55, 56, 63, 64, 65]
    offs = wl.packed_offsets(lens, align=16)
    host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    dev = torch.from_numpy(host).to(cuda)
    cut = (lens // 3).astype(np.int64)
    pre = [Sha1Ctx().update(host[int(o):int(o) + int(k)]) for o, k in zip(offs, cut)]
    states = torch.from_numpy(np.frombuffer(b"".join(p.raw() for p in pre), np.uint8).copy()).to(cuda)
    cio.sha1_update_batch_dev(dev, _dev_i64(offs.astype(np.int64) + cut, cuda),
                              _dev_i64(lens.astype(np.int64) - cut, cuda), states)
    raw = cio.sha1_states_view(states)["raw"]
    got = cio.sha1_final_batch_dev(states)
    for i in range(n):
        whole = host[int(offs[i]):int(offs[i] + lens[i])].tobytes()
        assert raw[i].tobytes() == Sha1Ctx().update(whole).raw(), i
        assert bytes(got[i]) == hashlib.sha1(whole).digest(), i


def test_device_contexts_against_openssl_fixtures(cuda):
    """tests/golden/sha1_ctx_vectors.json (libcrypto's SHA_CTX bytes after
    every piece, recorded by make_sha1_ctx.py): the same pieces fed through
    cio_sha1_update_batch_dev, one launch per piece over all 15 messages at
    once, leave exactly those bytes; the digests match too."""
    import json
    import os
    import torch
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sha1_ctx_vectors.json")) as f:
        g = json.load(f)
    cases = g["cases"]
    msgs = [wl.gen_chunk(g["seed"], c["id"], sum(c["pieces"])).tobytes() for c in cases]
    from test_gpu_crc import pack, to_dev
    buf, offs, _ = pack(msgs, misalign=[i % 16 for i in range(len(msgs))])
    dev = to_dev(buf, cuda)
    n = len(cases)
    states = cio.sha1_states_init(n, cuda)
    raw = cio.sha1_states_view(states)["raw"]
    assert [raw[i].tobytes().hex() for i in range(n)] == [c["ctx_after_each"][0] for c in cases]
    pos = np.zeros(n, np.int64)
    for k in range(max(len(c["pieces"]) for c in cases)):
        ln = np.array([c["pieces"][k] if k < len(c["pieces"]) else 0 for c in cases], np.int64)
        cio.sha1_update_batch_dev(dev, _dev_i64(offs.astype(np.int64) + pos, cuda), _dev_i64(ln, cuda), states)
        pos += ln
        raw = cio.sha1_states_view(states)["raw"]
        for i, c in enumerate(cases):
            if k < len(c["pieces"]):
                assert raw[i].tobytes().hex() == c["ctx_after_each"][k + 1], (c["id"], k)
    got = cio.sha1_final_batch_dev(states)
    assert [bytes(d).hex() for d in got] == [c["digest"] for c in cases]


def _geometry_check(n, seed, device="cuda"):
    """Two SHA1_Update batches (a random cut per chunk) over n ragged chunks at
    odd offsets, then SHA1_Final and the one-shot kernel: the number of mid
    contexts that differ from the host SHA-1's (OpenSSL's bytes) plus digests
    that differ from hashlib's."""
    import torch
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 2500, n).astype(np.uint64)
    offs = wl.packed_offsets(lens, align=1, start=5)
    host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    dev = torch.from_numpy(host).to(device)
    cut = (lens * rng.random(n)).astype(np.int64)
    states = cio.sha1_states_init(n, device)
    cio.sha1_update_batch_dev(dev, _dev_i64(offs, device), _dev_i64(cut, device), states)
    mid = cio.sha1_states_view(states)["raw"]
    cio.sha1_update_batch_dev(dev, _dev_i64(offs.astype(np.int64) + cut, device),
                              _dev_i64(lens.astype(np.int64) - cut, device), states)
    fin = cio.sha1_final_batch_dev(states)
    one = cio.sha1_batch_dev(dev, offs, lens)
    bad = 0
    for i in range(n):
        o, ln, c = int(offs[i]), int(lens[i]), int(cut[i])
        bad += mid[i].tobytes() != cio.Sha1().update(host[o:o + c]).state
        want = hashlib.sha1(host[o:o + ln].tobytes()).digest()
        bad += (bytes(fin[i]) != want) + (bytes(one[i]) != want)
    return bad


@pytest.mark.parametrize("per_wg", ["8", "16", "32"])
def test_every_geometry_continues_contexts(cuda, per_wg):
    """Each workgroup geometry of the SHA-1 kernel (8, 16 or 32 chunks per
    workgroup, forced with CIO_SHA1_CHUNKS_PER_WG under CIO_GPU_DIAG=1 in a
    process of its own: the choice is read once) over 700 ragged chunks at
    odd offsets: the mid-message contexts equal the host SHA-1's (OpenSSL's
    bytes), the finished digests and the one-shot digests equal hashlib's."""
    import os
    import subprocess
    import sys
    tests = os.path.dirname(os.path.abspath(__file__))
    code = (f"import sys; sys.path.insert(0, {os.path.dirname(tests)!r}); sys.path.insert(0, {tests!r}); "
            "import test_gpu_sha1 as t; print('bad', t._geometry_check(700, 86))")
    env = dict(os.environ, CIO_GPU_DIAG="1", CIO_SHA1_CHUNKS_PER_WG=per_wg)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "bad 0" in r.stdout, r.stdout


def test_wide_geometry_continues_contexts_in_process(cuda):
    """5000 chunks: more than 16 per CU, so the default 32-chunk geometry runs
    the continuation; mid contexts, finals and one-shot digests as above."""
    assert _geometry_check(5000, 87, cuda) == 0
