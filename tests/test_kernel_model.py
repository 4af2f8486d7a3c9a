"""CPU model of the GPU kernel's decomposition (host logic; no GPU).

Re-plays, in Python, exactly the work split of crc32_gpu.hip -- plan
construction (virtual aligned chunks, wave-steps, even split over W waves,
first chunk per wave), per-(sub-chain, lane) 16-byte blocks [1024 q + 16 lane, +16) with the
4080-byte step shift, head zeroing + seed fold (which can straddle lanes 0 and
1), partial last steps, per-sub-chain shift to the piece end,
piece slots (wave + chunk) and the finisher's Horner fold -- using the oracle
for the per-lane byte CRCs and GF(2) shifts.  Any index slip in that scheme
shows up here as a CRC mismatch against crc_update on the whole chunk.
"""
import numpy as np
import pytest

from oracle import pyoracle as po

STEP, GRAN, SUB, WAVE = 4096, 16, 4, 64
ROW = GRAN * WAVE
INIT = 0xFFFFFFFF


def plan(offs, lens, W):
    desc, S = [], 0
    for o, n in zip(offs, lens):
        h = o & 15
        vlen = h + n
        ns = (vlen + STEP - 1) // STEP if n >= 4 else 0
        desc.append(dict(a=o - h, h=h, vlen=vlen, g=S, nsteps=ns))
        S += ns
    wc, c = [], 0
    for w in range(W):
        g0 = (w * S) // W if S else 0
        while c < len(desc) and (desc[c]["nsteps"] == 0 or desc[c]["g"] + desc[c]["nsteps"] <= g0):
            c += 1
        wc.append(min(c, len(desc) - 1))
    return desc, S, wc


def lane_block(buf, d, jj, q, lane, seed):
    """Bytes of (sub-chain q, lane) at step jj (virtual chunk, head zeroed, seed folded)."""
    bstart = jj * STEP + q * ROW + lane * GRAN
    vb = 0 if bstart >= d["vlen"] else min(d["vlen"] - bstart, GRAN)
    blk = np.array(buf[d["a"] + bstart: d["a"] + bstart + vb], dtype=np.uint8)
    if jj == 0 and q == 0 and vb:
        sb = np.frombuffer(int(seed).to_bytes(4, "little"), np.uint8)
        for k in range(vb):
            pos = bstart + k                      # virtual position
            if pos < d["h"]:
                blk[k] = 0
            elif pos < d["h"] + 4:
                blk[k] ^= sb[pos - d["h"]]
    return bstart, vb, blk


def model(buf, offs, lens, seeds, W):
    desc, S, wc = plan(offs, lens, W)
    partials = {}
    start = lambda w: (w * S) // W  # noqa: E731
    for w in range(W):
        g, gend = start(w), start(w + 1)
        if g >= gend:
            continue
        c = wc[w]
        d = desc[c]
        j = g - d["g"]
        while True:
            jend = min(d["nsteps"], j + (gend - g))
            s = {}
            end = {}
            for jj in range(j, jend):
                for q in range(SUB):
                    for lane in range(WAVE):
                        bstart, vb, blk = lane_block(buf, d, jj, q, lane, seeds[c] if jj == 0 else 0)
                        if vb == 0:
                            continue
                        st = po.crc_shift(s.get((q, lane), 0), STEP - GRAN)   # step shift
                        s[(q, lane)] = po.crc_update(st, blk)
                        end[(q, lane)] = bstart + vb
            pend = min(jend * STEP, d["vlen"])
            acc = 0
            for key, st in s.items():
                if st:
                    dist = max(0, pend - end[key])
                    assert dist < 2 * STEP
                    acc ^= po.crc_shift(st, dist)
            slot = w + c
            assert slot not in partials
            partials[slot] = acc
            g += jend - j
            if g >= gend:
                break
            c += 1
            while desc[c]["nsteps"] == 0:
                c += 1
            d = desc[c]
            j = 0
    # finisher
    wave_of = lambda gg: ((gg + 1) * W + S - 1) // S - 1  # noqa: E731
    out = []
    for c, d in enumerate(desc):
        if d["nsteps"] == 0:
            out.append(po.crc_update(seeds[c], buf[offs[c]:offs[c] + lens[c]]))
            continue
        w0, w1 = wave_of(d["g"]), wave_of(d["g"] + d["nsteps"] - 1)
        acc = partials[w0 + c]
        for w in range(w0 + 1, w1 + 1):
            st, en = start(w), start(w + 1)
            if st == en:
                continue
            ps, pe = st - d["g"], min(en - d["g"], d["nsteps"])
            nb = d["vlen"] - ps * STEP if w == w1 else (pe - ps) * STEP
            acc = po.crc_shift(acc, nb) ^ partials[w + c]
        out.append(acc)
    return out


@pytest.mark.parametrize("W", [1, 3, 8, 64])
def test_model_matches_crc_update(W):
    rng = np.random.default_rng(W)
    lens = [0, 1, 3, 4, 5, 63, 64, 65, 4095, 4096, 4097, 8200, 13000, 2, 9000, 0, 30000]
    offs, pos = [], 0
    for n in lens:
        pos = ((pos + 15) & ~15) + int(rng.integers(0, 16))
        offs.append(pos)
        pos += n
    buf = rng.integers(0, 256, pos + 32, dtype=np.uint8)
    seeds = [int(x) for x in rng.integers(0, 2 ** 32, len(lens))]
    got = model(buf, offs, lens, seeds, W)
    want = [po.crc_update(s, buf[o:o + n]) for s, o, n in zip(seeds, offs, lens)]
    assert got == want


def _layout(offs, lens, W):
    import ctypes
    from chunkio_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    f = lib.cioa_debug_plan_layout
    u64p = ctypes.POINTER(ctypes.c_uint64)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    f.argtypes = [u64p, u64p, ctypes.c_size_t, ctypes.c_uint32, u32p, u32p]
    o = np.ascontiguousarray(offs, np.uint64)
    n_ = np.ascontiguousarray(lens, np.uint64)
    cw = np.zeros(3 * len(o), np.uint32)
    wf = np.zeros(W, np.uint32)
    assert f(o.ctypes.data_as(u64p), n_.ctypes.data_as(u64p), len(o), W,
             cw.ctypes.data_as(u32p), wf.ctypes.data_as(u32p)) == 0
    return cw.reshape(-1, 3), wf


@pytest.mark.parametrize("W,kind", [(4096, "cfg2"), (4096, "mixed"), (4096, "fewer_steps"), (256, "mixed"), (48, "mixed")])
def test_plan_workgroup_local_fold_flags(W, kind):
    """The C plan's per-chunk wave range (w0, w1) and per-wave LDS-fold flags
    (crc32_gpu.hip plan_build) against a restatement of their definition:
    a split chunk whose first and last piece lie in one 16-wave workgroup is
    folded by the wave holding its final piece (bit 0, bits 8.. = waves
    before it), and every earlier wave ending inside it hands its piece over
    (bit 1); all other split chunks take the global arrival."""
    rng = np.random.default_rng(W + len(kind))
    if kind == "cfg2":
        lens = np.full(1024, 409600, np.uint64)
    elif kind == "mixed":
        lens = rng.integers(1, 3 << 20, 3000).astype(np.uint64)
        lens[::7] = rng.integers(0, 4, lens[::7].size)
    else:
        lens = rng.integers(1, 40000, 40).astype(np.uint64)   # S < W: empty wave ranges
    offs = np.cumsum(np.concatenate([[5], lens[:-1] + 3])).astype(np.uint64)
    if kind == "cfg2":
        offs = np.arange(1024, dtype=np.uint64) * np.uint64(409600)
    desc, S, wc = plan(list(map(int, offs)), list(map(int, lens)), W)
    cw, wf = _layout(offs, lens, W)
    start = lambda w: (w * S) // W  # noqa: E731
    wave_of = lambda gg: ((gg + 1) * W + S - 1) // S - 1  # noqa: E731
    local = {}
    for c, d in enumerate(desc):
        if d["nsteps"] == 0:
            continue
        w0, w1 = wave_of(d["g"]), wave_of(d["g"] + d["nsteps"] - 1)
        assert (cw[c, 0], cw[c, 1]) == (w0, w1), c
        npieces = sum(1 for w in range(w0, w1 + 1) if start(w) < start(w + 1))
        assert cw[c, 2] == npieces, c
        local[c] = npieces > 1 and w0 // 16 == w1 // 16
    n_fold = n_pub = 0
    for w in range(W):
        g0, g1 = start(w), start(w + 1)
        want = 0
        if g0 < g1:
            first = desc[wc[w]]
            if first["g"] < g0 and first["g"] + first["nsteps"] <= g1 and local[wc[w]]:
                want |= 1 | ((w - wave_of(first["g"])) << 8)
            cl = max(c for c, d in enumerate(desc) if d["nsteps"] and d["g"] < g1)
            if desc[cl]["g"] + desc[cl]["nsteps"] > g1 and local[cl]:
                want |= 2
        assert wf[w] == want, w
        n_fold += want & 1
        n_pub += (want >> 1) & 1
    assert n_fold == sum(local.values())
    if kind == "cfg2":
        # 100-step chunks, 25 steps per wave: every chunk is split over 4
        # waves of one workgroup.
        assert n_fold == 1024 and n_pub == 3 * 1024
