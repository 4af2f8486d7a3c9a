#!/usr/bin/env python3
"""Generates chunkio_amd/csrc/sha1_wave_rounds.inc: the round wave of
sha1_wave_kernel (chunkio_amd/csrc/sha1_gpu.hip) as one inline-asm routine.

Why asm: the round wave keeps K_t + W_t in SGPRs, loaded by s_load_dwordx16
while earlier rounds run.  Scalar loads land asynchronously, and with the
loads in separate inline-asm statements the compiler moved in-flight SGPRs
between statements (a phi copy before the wait).  One asm routine owns its
SGPRs (clobbered) from load to wait, so nothing reads them early.

    python tools/gen_sha1_wave_asm.py > chunkio_amd/csrc/sha1_wave_rounds.inc

Rows: a pass's K + W words of one chunk are one stream (block j's 80 words at
word 80 j) in the chunk's region of the ring slot, followed by PAD_BYTES of
readable padding.  The stream is consumed in 32-word segments, each two
s_load_dwordx16 (glc: the slot held an older pass) into one of two 32-SGPR
buffers; segment k + 1 is requested when segment k's wait is over, so a load
has 32 rounds (~650 cycles) to land: with 16-word segments the waits cost
~315 cycles each (profiles/r03/sha1/ab_sha1_wave16_*).  Scalar loads may
return out of order, so every wait is lgkmcnt(0).  The routine walks 4
blocks (10 segments) per loop turn from one base pointer (immediate
offsets), leaving after any block once the pass's blocks are done.

Round t (FIPS 180-4 §6.1.2) with the registers renamed instead of moved: the
new a goes into the register of e, b is rotated in place, and the names shift
(a, b, c, d, e) -> (e, a, b, c, d), back to the start after 5 rounds:
    v_bitop3_b32   T, b, c, d            f_t (Ch / Parity / Maj)
    v_add_u32      e, s[K_t + W_t], e
    v_alignbit_b32 R, a, a, 27           rotl(a, 5)
    v_add3_u32     e, R, T, e
    v_alignbit_b32 b, b, b, 2            rotl(b, 30)
Five VALU per round.  A block starts from the chaining value H (h0..h4, never
written by the rounds): each state register's first write goes to the block's
own register X instead, reading H, so a block ends with H += X (5 adds) and
no copies.
"""

# Two 40-word SGPR buffers, each three scalar loads (x16, x16, x8).  Not
# contiguous: s32-s34 are the ABI's reserved stack/frame/base pointers.
BUFS = (((0, 16), (16, 16), (36, 8)), ((44, 16), (60, 16), (76, 8)))
SEG_WORDS = 40                       # a block is two segments
BLOCK_WORDS = 80
BLOCK_BYTES = BLOCK_WORDS * 4
SLOT_BYTES = 16 * BLOCK_BYTES        # kWvBlocks blocks of a chunk in one ring slot
NSLOTS = 3
PAD_BYTES = 256                      # readable padding after slot 2 (the last prefetch)
CHAIN_STRIDE = NSLOTS * SLOT_BYTES + PAD_BYTES   # a chunk's three slots, consecutive

F = {0: "0xca", 1: "0x96", 2: "0xe8", 3: "0x96"}   # Ch, Parity, Maj, Parity (bitop3 tables)

# bookkeeping SGPRs (clobbered with the buffers)
S_PASS, S_SLOT, S_NBP, S_CARRY = "s84", "s85", "s86", "s87"
S_LEFT = ("s88", "s89")              # blocks left (64-bit)
S_PTR = "s[90:91]"                   # the current block's rows
S_PTR_LO, S_PTR_HI = "s90", "s91"
CLOBBER = list(range(0, 32)) + list(range(36, 92))


def sreg(buf, i):
    for base, cnt in BUFS[buf]:
        if i < cnt:
            return f"s{base + i}"
        i -= cnt
    raise ValueError


def load_seg(lines, buf, off):
    for base, cnt in BUFS[buf]:
        lines.append(f"s_load_dwordx{cnt} s[{base}:{base + cnt - 1}], {S_PTR}, {hex(off)} glc")
        off += 4 * cnt


def block(lines):
    """One block from S_PTR: on entry segment 0 (buffer 0) is in flight; on
    exit the next block's segment 0 (S_PTR + 320, buffer 0) is."""
    cur = {k: f"%[h{k}]" for k in range(5)}
    xreg = {k: f"%[x{k}]" for k in range(5)}
    names = [0, 1, 2, 3, 4]
    for seg in range(2):
        lines.append("s_waitcnt lgkmcnt(0)")
        load_seg(lines, 1 - seg, (seg + 1) * SEG_WORDS * 4)
        for i in range(SEG_WORDS):
            t = seg * SEG_WORDS + i
            sa, sb, sc, sd, se = names
            lines.append(f"v_bitop3_b32 %[t], {cur[sb]}, {cur[sc]}, {cur[sd]} bitop3:{F[t // 20]}")
            lines.append(f"v_add_u32_e32 {xreg[se]}, {sreg(seg, i)}, {cur[se]}")
            cur[se] = xreg[se]
            lines.append(f"v_alignbit_b32 %[r], {cur[sa]}, {cur[sa]}, 27")
            lines.append(f"v_add3_u32 {cur[se]}, %[r], %[t], {cur[se]}")
            lines.append(f"v_alignbit_b32 {xreg[sb]}, {cur[sb]}, {cur[sb]}, 2")
            cur[sb] = xreg[sb]
            names = [se, sa, sb, sc, sd]
    assert names == [0, 1, 2, 3, 4] and all(cur[k] == xreg[k] for k in range(5))
    for k in range(5):
        lines.append(f"v_add_u32_e32 %[h{k}], %[h{k}], {xreg[k]}")


def routine():
    L = []
    L.append("s_barrier")                              # barrier 0: passes 0 and 1 published
    L.append(f"s_mov_b32 {S_PASS}, 0")
    L.append(f"s_mov_b32 {S_LEFT[0]}, %[nblo]")
    L.append(f"s_mov_b32 {S_LEFT[1]}, %[nbhi]")
    L.append(f"s_mov_b32 {S_SLOT}, 0")                 # ring slot = pass % 3
    L.append(f"s_mov_b32 {S_CARRY}, 0")                # 1: the next segment is in flight
    L.append("s_cmp_eq_u32 %[npass], 0")
    L.append("s_cbranch_scc1 .Lend%=")
    L.append(".Lpass%=:")
    L.append(f"s_cmp_eq_u32 {S_LEFT[1]}, 0")           # nbp = min(left, 16)
    L.append(f"s_cselect_b32 {S_NBP}, {S_LEFT[0]}, 16")
    L.append(f"s_min_u32 {S_NBP}, {S_NBP}, 16")
    L.append(f"s_sub_u32 {S_LEFT[0]}, {S_LEFT[0]}, {S_NBP}")
    L.append(f"s_subb_u32 {S_LEFT[1]}, {S_LEFT[1]}, 0")
    L.append(f"s_mul_i32 {S_PTR_HI}, {S_SLOT}, {SLOT_BYTES}")
    L.append(f"s_add_u32 {S_PTR_LO}, %[blo], {S_PTR_HI}")
    L.append(f"s_addc_u32 {S_PTR_HI}, %[bhi], 0")
    L.append(f"s_cmp_eq_u32 {S_NBP}, 0")
    L.append("s_cbranch_scc1 .Lsettle%=")              # no block: settle a carried load
    L.append(f"s_cmp_eq_u32 {S_CARRY}, 1")
    L.append("s_cbranch_scc1 .Lturn%=")
    load_seg(L, 0, 0)
    L.append(".Lturn%=:")
    for u in range(2):                                 # two blocks per loop turn
        block(L)
        L.append(f"s_add_u32 {S_PTR_LO}, {S_PTR_LO}, {BLOCK_BYTES}")
        L.append(f"s_addc_u32 {S_PTR_HI}, {S_PTR_HI}, 0")
        L.append(f"s_sub_u32 {S_NBP}, {S_NBP}, 1")
        L.append(f"s_cmp_eq_u32 {S_NBP}, 0")
        L.append("s_cbranch_scc1 .Ldone%=")
    L.append("s_branch .Lturn%=")
    L.append(".Ldone%=:")
    # The load past the pass's last block reads the next slot's first segment
    # unless the slot is the last (then the padding): the chunk's slots are
    # consecutive, and pass p + 1 was published at barrier p, so that is the
    # next pass's first segment whenever the next pass has blocks of this chunk
    # (this pass then had all 16).  Keep it in flight across the barrier; a
    # next pass without blocks settles it.
    L.append(f"s_cmp_eq_u32 {S_SLOT}, 2")
    L.append("s_cbranch_scc1 .Lsettle%=")
    L.append(f"s_mov_b32 {S_CARRY}, 1")
    L.append("s_branch .Lbar%=")
    L.append(".Lsettle%=:")
    L.append("s_waitcnt lgkmcnt(0)")
    L.append(f"s_mov_b32 {S_CARRY}, 0")
    L.append(".Lbar%=:")
    L.append("s_barrier")                              # barrier pass + 1
    L.append(f"s_add_u32 {S_PASS}, {S_PASS}, 1")
    L.append(f"s_add_u32 {S_SLOT}, {S_SLOT}, 1")
    L.append(f"s_cmp_eq_u32 {S_SLOT}, 3")
    L.append(f"s_cselect_b32 {S_SLOT}, 0, {S_SLOT}")
    L.append(f"s_cmp_lt_u32 {S_PASS}, %[npass]")
    L.append("s_cbranch_scc1 .Lpass%=")
    L.append("s_waitcnt lgkmcnt(0)")                   # nothing may stay in flight past the routine
    L.append(".Lend%=:")
    return L


DIAG = set()   # A/B diagnostics (wrong digests): "nowait", "noload", "noglc", "exec=<mask>"


def main():
    import sys
    DIAG.update(a for a in sys.argv[1:])
    L = routine()
    if "nowait" in DIAG:   # timing only: rounds use SGPRs whose loads may not have landed
        # (the waits before the barrier branch and at the exit stay: no load
        # may land after the routine, in SGPRs the compiler uses again)
        keep = {L.index(".Ldone%=:") + 1, len(L) - 2}
        L = [l for i, l in enumerate(L) if l != "s_waitcnt lgkmcnt(0)" or i in keep]
        i = L.index(".Ldone%=:")
        L[i + 1:i + 1] = [] if L[i + 1] == "s_waitcnt lgkmcnt(0)" else ["s_waitcnt lgkmcnt(0)"]
        L.insert(L.index("s_branch .Lbar%="), "s_waitcnt lgkmcnt(0)")
    if "noload" in DIAG:   # timing only: no scalar loads or waits at all (the rounds' issue floor)
        L = [l for l in L if not l.startswith("s_load_") and l != "s_waitcnt lgkmcnt(0)"]
    if "noglc" in DIAG:    # timing only: scalar-cache hits allowed (stale rows possible)
        L = [l.replace(" glc", "") for l in L]
    for d in DIAG:
        if d.startswith("exec="):   # run the rounds on fewer lanes (lane 0 holds the result)
            L = [f"s_mov_b64 s[92:93], exec", f"s_mov_b64 exec, {d[5:]}"] + L + ["s_mov_b64 exec, s[92:93]"]
            CLOBBER.extend([92, 93])
    print("// Generated by tools/gen_sha1_wave_asm.py -- do not edit.")
    print("// The round wave of sha1_wave_kernel: every pass's blocks of one chunk,")
    print("// K + W from SGPRs (see the generator's docstring).  Operands: h0..h4")
    print("// (chaining value, in/out), x0..x4, t, r (scratch VGPRs), blo/bhi (the")
    print("// chunk's rows in ring slot 0), npass, nblo/nbhi (the chunk's block count).")
    print(f"#define CIOA_SHA1_WAVE_CHAIN_STRIDE {CHAIN_STRIDE}   // bytes per chunk: its {NSLOTS} ring slots + padding")
    print(f"#define CIOA_SHA1_WAVE_SLOT_BYTES {SLOT_BYTES}      // one slot: a pass's {SLOT_BYTES // BLOCK_BYTES} blocks of rows")
    print("#define CIOA_SHA1_WAVE_ROUNDS_ASM \\")
    for l in L:
        print(f'    "{l}\\n" \\')
    print('    ""')
    print("#define CIOA_SHA1_WAVE_ROUNDS_CLOBBERS \\")
    regs = ", ".join(f'"s{k}"' for k in CLOBBER)
    print(f"    {regs}, \"scc\", \"memory\"")


if __name__ == "__main__":
    main()
