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


def head_align():
    """The library's virtual-start alignment for chunks longer than one step
    (CIO_HEAD_ALIGN, reported in cio_gpu_version: 16 or 128)."""
    import re
    import chunkio_amd
    m = re.search(rb"head-align=(\d+)", chunkio_amd.lib().cio_gpu_version())
    return int(m.group(1)) if m else 16


def plan(offs, lens, W, align=None):
    align = head_align() if align is None else align
    desc, S = [], 0
    for o, n in zip(offs, lens):
        h = o & ((align - 1) if n > STEP else 15)
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


def model(buf, offs, lens, seeds, W, align=None):
    desc, S, wc = plan(offs, lens, W, align)
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


@pytest.mark.parametrize("align", [16, 128])
@pytest.mark.parametrize("W", [1, 3, 8, 64])
def test_model_matches_crc_update(W, align):
    rng = np.random.default_rng(W)
    lens = [0, 1, 3, 4, 5, 63, 64, 65, 4095, 4096, 4097, 8200, 13000, 2, 9000, 0, 30000]
    offs, pos = [], 0
    for n in lens:
        pos = ((pos + 15) & ~15) + int(rng.integers(0, 16))
        offs.append(pos)
        pos += n
    buf = rng.integers(0, 256, pos + 32, dtype=np.uint8)
    seeds = [int(x) for x in rng.integers(0, 2 ** 32, len(lens))]
    got = model(buf, offs, lens, seeds, W, align)
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


# ---- L64 layout (issue-ahead kernel, CIO_GPU_L64): one chain per lane -------

def _permlane16_swap(a, b):
    """v_permlane16_swap_b32 a, b: odd 16-lane rows of a <-> even rows of b."""
    a, b = a.copy(), b.copy()
    for r in (0, 2):
        lo, hi = slice(16 * r, 16 * r + 16), slice(16 * (r + 1), 16 * (r + 2))
        a[hi], b[lo] = b[lo].copy(), a[hi].copy()
    return a, b


def _permlane32_swap(a, b):
    """v_permlane32_swap_b32 a, b: lanes 32..63 of a <-> lanes 0..31 of b."""
    a, b = a.copy(), b.copy()
    a[32:], b[:32] = b[:32].copy(), a[32:].copy()
    return a, b


def test_l64_transpose_gives_each_lane_64_contiguous_bytes():
    """Row r's load gives lane (g, i) = 16 g + i the block 4 i + g of row r;
    the two butterfly stages of load_step64/transpose64 then leave register
    k of lane L holding step bytes [64 L + 16 k, +16).  Modelled on block
    indices (one 'dword' per block)."""
    lane = np.arange(64)
    regs = [r * 64 + 4 * (lane & 15) + (lane >> 4) for r in range(4)]   # block index in the step
    regs[0], regs[1] = _permlane16_swap(regs[0], regs[1])
    regs[2], regs[3] = _permlane16_swap(regs[2], regs[3])
    regs[0], regs[2] = _permlane32_swap(regs[0], regs[2])
    regs[1], regs[3] = _permlane32_swap(regs[1], regs[3])
    for k in range(4):
        np.testing.assert_array_equal(regs[k], 4 * lane + k)
    # every load instruction still reads one whole 1 KiB row
    for r in range(4):
        offs = r * 1024 + 64 * (lane & 15) + 16 * (lane >> 4)
        assert sorted(offs.tolist()) == list(range(r * 1024, r * 1024 + 1024, 16))


@pytest.mark.parametrize("nsteps,seed", [(1, INIT), (3, 0x1234ABCD), (25, INIT)])
def test_l64_chain_decomposition(nsteps, seed):
    """One chain per lane over [64 L, 64 L + 64) of every step, a 4032-byte
    shift between steps, the seed on content bytes 0..3, the piece end
    reached by x^(8 * 64 (63 - L)) and an XOR over the wave: equals
    crc_update over the whole (aligned, whole-step) chunk."""
    rng = np.random.default_rng(nsteps)
    data = rng.integers(0, 256, nsteps * STEP, dtype=np.uint8)
    acc = 0
    for L in range(WAVE):
        s = 0
        for j in range(nsteps):
            blk = data[j * STEP + 64 * L: j * STEP + 64 * L + 64].copy()
            if j == 0 and L == 0:
                blk[:4] ^= np.frombuffer(int(seed).to_bytes(4, "little"), np.uint8)
            s = po.crc_update(po.crc_shift(s, STEP - 64), blk)
        acc ^= po.crc_shift(s, 64 * (63 - L))
    assert acc == po.crc_update(seed, data)
