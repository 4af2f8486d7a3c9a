// crc32_gpu.hip -- batched CRC-32 over independent chunk content buffers,
// hand-written for CDNA4 (gfx950, MI355X).  C ABI in
// include/chunkio_amd/cio_crc32_gpu.h.
//
// Reference behaviour reproduced (fluent/chunkio):
//   crc_update(state, buf, len)  deps/crc32/crc32.c:337-390 — CRC-32/IEEE,
//   reflected poly 0xEDB88320, raw (un-finalized) state in and out.  Each
//   chunk i of a batch yields crc_update(seed_i, base + off_i, len_i), i.e.
//   cio_file_calculate_checksum() (src/cio_file.c:66-94) over that chunk.
//
// Algorithm (see DESIGN.md for the derivation and the roofline):
//   The CRC is affine over GF(2):  crc(s, A||B) = shift(crc(s, A), |B|) ^
//   crc(0, B), shift(s, n) = s * x^(8n) mod P.  Every chunk is cut into
//   4 KiB wave-steps; step j of a chunk covers virtual bytes [4096 j, 4096 j
//   + 4096) where the virtual chunk is the content prefixed by its (off & 15)
//   misalignment bytes, which are zeroed (a zero-seeded CRC ignores leading
//   zeros) so every load is an aligned 16-byte global_load_dwordx4.  A step
//   is 4 coalesced 1 KiB rows; lane l runs 4 sub-chains, sub-chain q over the
//   16 bytes [1024 q + 16 l, +16) of every step, slice-by-4 with lookup tables
//   held in LDS, replicated 32 times so lane l always hits bank (l & 31): no
//   data-dependent bank conflicts.  Between two steps a sub-chain jumps the
//   4080 bytes to its next block (one 4-lookup shift table).  The seed is
//   folded into the first 4 content bytes.  At the end of a piece (the steps
//   of one chunk that one wave owns) the sub-chains are shifted to the piece
//   end (Horner over q + one lane factor) and the wave XOR-reduces with
//   __shfl_xor.  A whole-chunk piece is the chunk's CRC; otherwise the last
//   wave to publish a piece of the chunk folds the pieces -> one raw CRC per
//   chunk.  Batches of chunks <= 4 KiB use crc32_small_kernel instead.
//
//   Work partition: the S wave-steps of the whole batch are split evenly over
//   the W persistent waves of the grid (one 1024-thread workgroup per CU), so
//   every wave streams the same number of bytes whatever the chunk sizes —
//   the load-balanced persistent kernel of BASELINE config 3.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <vector>
#include <string>
#include <algorithm>

#include <type_traits>

#include "cio_gpu_internal.h"

using namespace cioa;

namespace {

// ---------------------------------------------------------------- device math

// Compile-time GF(2) arithmetic (same math as crc32_host.c) for table constants.
constexpr uint32_t cx_multmodp(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
    for (int i = 31; i >= 0; --i) {
        if ((a >> i) & 1u) {
            p ^= b;
        }
        b = (b & 1u) ? (b >> 1) ^ CIOA_POLY : (b >> 1);
    }
    return p;
}

constexpr uint32_t cx_xpow8n(uint64_t n)
{
    uint32_t r = 0x80000000u, sq = 0x00800000u;
    while (n) {
        if (n & 1u) {
            r = cx_multmodp(sq, r);
        }
        sq = cx_multmodp(sq, sq);
        n >>= 1;
    }
    return r;
}

// a(x) * b(x) mod P(x), reflected bit order (bit 31 = x^0).
__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
#pragma unroll
    for (int i = 31; i >= 0; --i) {
        p ^= b & (0u - ((a >> i) & 1u));
        b = (b >> 1) ^ (CIOA_POLY & (0u - (b & 1u)));
    }
    return p;
}

// b(x) * C(x) mod P for a compile-time C: linear in the 32 bits of b, so the
// XOR of the images of b's set bits (32 constants, no loop-carried shifts).
template <uint32_t C>
struct MulCols {
    uint32_t v[32];
    constexpr MulCols() : v{}
    {
        for (int j = 0; j < 32; ++j) {
            v[j] = cx_multmodp(C, 1u << j);
        }
    }
};

// One v_bfe_i32 (the bit as a 0 / ~0 mask) and one v_bitop3_b32 (x ^ (m & c))
// per bit into four accumulators: 66 instructions without a loop-carried
// shift, ~0.15 us for a wave alone against ~0.4 us for multmodp
// (tools/probe/gf2_probe.hip) -- the fold at a wave's range end runs while
// the rest of the CU may be idle.
template <uint32_t C>
__device__ __forceinline__ uint32_t mulconst(uint32_t b)
{
    constexpr MulCols<C> K;
    uint32_t p[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        p[j & 3] = __builtin_amdgcn_bitop3_b32(p[j & 3], 0u - ((b >> j) & 1u), K.v[j], 0x78);
    }
    return __builtin_amdgcn_bitop3_b32(p[0], p[1], p[2], 0x96) ^ p[3];
}

// Sub-chain states of a lane whose last step was full, shifted to the lane's
// row end and XORed: sum_q s_q x^(8 * 1024 (3 - q)), by Horner.  TREE: the
// bit-column form (fewer instructions in a row: uniform batches end all their
// pieces together at the kernel's end, where one wave's latency counts); the
// shift-chain form measured 0.2% faster where pieces end mid-stream among
// streaming waves (cfg3, profiles/r02/ab_lds_fold_preshifted.txt).
template <bool TREE>
__device__ __forceinline__ uint32_t fold_full(const uint32_t (&s)[kSub])
{
    constexpr uint32_t kXRow = cx_xpow8n(kRow);
    uint32_t h = s[0];
#pragma unroll
    for (int q = 1; q < kSub; ++q) {
        h = (TREE ? mulconst<kXRow>(h) : multmodp(kXRow, h)) ^ s[q];
    }
    return h;
}

// floor(x / d) for x < 2^52, d >= 1: a correctly rounded double quotient is
// within one of the integer quotient (x and d are exact in a double), and one
// compare-and-step fixes it.  A 64-bit integer division is a ~120-instruction
// SALU routine for wave-uniform operands; at kernel start 16 waves per CU
// running three of them on the CU's one scalar unit delayed the last wave's
// first HBM request by ~2.5 us.  This is ~20 VALU instructions per wave.
__device__ __forceinline__ uint64_t div_u52(uint64_t x, uint64_t d)
{
    uint64_t q = (uint64_t) ((double) x / (double) d);
    if (q * d > x) {
        q -= 1;
    } else if ((q + 1) * d <= x) {
        q += 1;
    }
    return q;
}

__device__ __forceinline__ uint64_t uniform_u64(uint64_t v)
{
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t) v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t) (v >> 32));
    return ((uint64_t) hi << 32) | lo;
}

// floor(w * X / W), the even split of X units over W waves.  The plan
// guarantees S < 2^40 and W <= 2^12 (plan_create), so w * X < 2^52.  A full
// MI355X has W = 256 x 16 = 2^12 waves: then it is a uniform multiply and
// shift on the scalar unit, and the kernels' first HBM requests wait on no
// floating-point division.
__device__ __forceinline__ uint64_t split_point(uint64_t w, uint64_t X, uint64_t W)
{
    if ((W & (W - 1)) == 0) {
        return (w * X) >> __builtin_ctzll(W);
    }
    return div_u52(w * X, W);
}

__device__ __forceinline__ uint64_t wave_start(uint64_t w, uint64_t S, uint64_t W)
{
    return split_point(w, S, W);
}

// Replicas the lookups use: 32 slice / 8 shift.  Diagnostic build
// (-DCIO_DIAG_HALF_REPLICAS): lanes read only 16 slice and 4 shift replicas
// -- the tables a workgroup would hold in half the LDS (80 KiB, two
// workgroups per CU) -- so every lookup group of 32 lanes takes the 2-way
// bank conflicts such a layout has, at the current occupancy.
#if CIO_DIAG_HALF_REPLICAS
constexpr uint32_t kSliceRepMask = 15u, kShiftRepMask = 3u;
#else
constexpr uint32_t kSliceRepMask = 31u, kShiftRepMask = 7u;
#endif

// Slice tables in LDS, replicated 32x so lane l always reads bank (l & 31):
//   byte address(k, b, lane) = (k>>1)*65536 + b*256 + (k&1)*128 + (lane&31)*4
// One v_perm_b32 builds the address: {0, k>>1, x.byte, lane*4}.  lbase_hi =
// lane*4 | 0x10000 selects tables 2-3, lbase_lo = lane*4 tables 0-1; (k&1)*128
// is the instruction's immediate offset.
template <int K>
__device__ __forceinline__ uint32_t tl(const char *lds, uint32_t lbase, uint32_t x, int byte)
{
    const uint32_t sel = 0x0c020000u | ((4u + (uint32_t) byte) << 8);
    const uint32_t addr = __builtin_amdgcn_perm(x, lbase, sel);
    return *reinterpret_cast<const uint32_t *>(lds + addr + ((K & 1) << 7));
}

// crc_update(s, 4 little-endian bytes of w):
//   s' = T3[x.b0] ^ T2[x.b1] ^ T1[x.b2] ^ T0[x.b3],  x = s ^ w,  Tk = shift by k+1 bytes
__device__ __forceinline__ uint32_t word_step(const char *lds, uint32_t lb_lo, uint32_t lb_hi,
                                              uint32_t s, uint32_t w)
{
    const uint32_t x = s ^ w;
    return tl<3>(lds, lb_hi, x, 0) ^ tl<2>(lds, lb_hi, x, 1) ^
           tl<1>(lds, lb_lo, x, 2) ^ tl<0>(lds, lb_lo, x, 3);
}

__device__ __forceinline__ uint32_t byte_step(const char *lds, uint32_t lb_lo, uint32_t s, uint32_t byte)
{
    return tl<0>(lds, lb_lo, (s ^ byte) & 0xffu, 0) ^ (s >> 8);
}

// shift(s, kStep - kGran): jump a sub-chain over the 4080 bytes between its
// 16-byte blocks in consecutive steps.  8 replicas: address k*8192 + b*32 + (lane&7)*4.
__device__ __forceinline__ uint32_t step_shift(const char *lds, uint32_t lrep, uint32_t s)
{
    const char *t = lds + kShiftOff + lrep;
    return __builtin_amdgcn_bitop3_b32(*reinterpret_cast<const uint32_t *>(t + (s & 0xffu) * 32u),
                                       *reinterpret_cast<const uint32_t *>(t + 8192 + ((s >> 8) & 0xffu) * 32u),
                                       *reinterpret_cast<const uint32_t *>(t + 16384 + ((s >> 16) & 0xffu) * 32u),
                                       0x96) ^
           *reinterpret_cast<const uint32_t *>(t + 24576 + (s >> 24) * 32u);
}

// a ^ b ^ c in one gfx950 v_bitop3_b32.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// The steady-state step of one sub-chain: shift(s, 4080) then crc_update over
// the 16 bytes of v.  The four lookups of every word and the next data word
// are combined with two 3-input XORs (10 XOR instructions per 16 bytes
// instead of 19).
// crc_update(h, the 16 bytes of v): four dependent rounds of four lookups.
__device__ __forceinline__ uint32_t block16(const char *lds, uint32_t lb_lo, uint32_t lb_hi, uint32_t h,
                                            const uint4 &v)
{
    uint32_t x = h ^ v.x;
    const uint32_t w[3] = {v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        x = xor3(xor3(tl<3>(lds, lb_hi, x, 0), tl<2>(lds, lb_hi, x, 1), tl<1>(lds, lb_lo, x, 2)),
                 tl<0>(lds, lb_lo, x, 3), w[i]);
    }
    return xor3(tl<3>(lds, lb_hi, x, 0), tl<2>(lds, lb_hi, x, 1), tl<1>(lds, lb_lo, x, 2)) ^
           tl<0>(lds, lb_lo, x, 3);
}

__device__ __forceinline__ uint32_t shift_block16(const char *lds, uint32_t lb_lo, uint32_t lb_hi,
                                                  uint32_t lrep, uint32_t s, const uint4 &v)
{
    return block16(lds, lb_lo, lb_hi, step_shift(lds, lrep, s), v);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Streaming loads: non-temporal (read once).  With the coalesced layout (a
// wave-instruction reads 1 KiB contiguous) this is the fastest HBM read
// policy measured on MI355X (tools/probe/crc_probe.hip).
__device__ __forceinline__ uint4 ldg16(const uint8_t *p)
{
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

// In-kernel table entries (no global memory on the start-up path):
//   slice table k, entry b = shift(b, k + 1)          (b advanced k+1 zero bytes)
//   shift table k, entry b = shift(b << 8k, kStep - kGran)
// Both are GF(2)-linear in the 8 bits of b, so an entry is the XOR of the
// images of b's set bits: 8 compile-time constants per table (immediates).
struct Basis8 {
    uint32_t v[8];
    constexpr Basis8(uint32_t mul, int byte_pos) : v{}
    {
        for (int j = 0; j < 8; ++j) {
            v[j] = cx_multmodp(mul, (1u << j) << (8 * byte_pos));
        }
    }
};

template <uint32_t MUL, int BYTE>
__device__ __forceinline__ uint32_t basis_entry(uint32_t b)
{
    constexpr Basis8 B(MUL, BYTE);
    uint32_t p = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        p ^= B.v[j] & (0u - ((b >> j) & 1u));
    }
    return p;
}

constexpr uint32_t kXStepShift = cx_xpow8n(kStep - kGran);

// SHIFT = x^(8 d) of the shift table's jump d (kStep - kGran for the stream
// kernel, kRow - kGran for the small-chunk kernel).
template <uint32_t SHIFT = kXStepShift>
__device__ __forceinline__ void table_entries(uint32_t k, uint32_t b, uint32_t &slice, uint32_t &shift)
{
    switch (k) {
    case 0: slice = basis_entry<cx_xpow8n(1), 0>(b); shift = basis_entry<SHIFT, 0>(b); break;
    case 1: slice = basis_entry<cx_xpow8n(2), 0>(b); shift = basis_entry<SHIFT, 1>(b); break;
    case 2: slice = basis_entry<cx_xpow8n(3), 0>(b); shift = basis_entry<SHIFT, 2>(b); break;
    default: slice = basis_entry<cx_xpow8n(4), 0>(b); shift = basis_entry<SHIFT, 3>(b); break;
    }
}

// Tables.  Thread tid owns entry b = tid & 255 of slice table k = tid >> 8
// (and of shift table k): the 1024 threads of the workgroup hold the 4 x 256
// entries exactly once.  Each replicated row of an entry is contiguous in
// the LDS images -- 32 replicas = 128 B of the slice image, 8 replicas =
// 32 B of the shift image -- so the thread writes its own rows directly:
// 8 + 2 ds_write_b128, no compact staging arrays, no gather, one barrier
// (by the caller).  Lane l writes granule (l + i) & 7 of its row in store i,
// so the 8 lanes of a ds_write_b128 lane group hit 8 different granules of
// their 256 B-strided rows: conflict-free.
constexpr int kE = 1024 / kThreads;            // table entries per thread
static_assert(kE == 1, "one slice and one shift entry per thread");

template <bool STAMPS = false, bool SHIFT = true>
__device__ __forceinline__ void write_tables(char *lds, uint32_t tid, const uint32_t (&tab_v)[kE],
                                             const uint32_t (&tab_sv)[kE], unsigned long long *ts = nullptr)
{
    const uint32_t k = tid >> 8, b = tid & 255u, lane = tid & 63u;
    const uint32_t srow = (k >> 1) * 65536u + b * 256u + (k & 1u) * 128u;
    const uint4 sv = make_uint4(tab_v[0], tab_v[0], tab_v[0], tab_v[0]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        *reinterpret_cast<uint4 *>(lds + srow + 16u * ((lane + (uint32_t) i) & 7u)) = sv;
    }
    if (SHIFT) {
        const uint32_t hrow = kShiftOff + k * 8192u + b * 32u;
        const uint4 hv = make_uint4(tab_sv[0], tab_sv[0], tab_sv[0], tab_sv[0]);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            *reinterpret_cast<uint4 *>(lds + hrow + 16u * ((lane + (uint32_t) i) & 1u)) = hv;
        }
    }
    if (STAMPS) {
        ts[0] = __builtin_amdgcn_s_memrealtime();
        ts[1] = ts[0];
    }
}

// One lane's 4 x 16 bytes of a step: sub-chain q holds [1024 q + 16 lane, +16).
struct StepRegs {
    uint4 q[kSub];
};

// Issue the 4 coalesced 16-byte loads of lane `lane` for step jj of a chunk.
// Each granule address is clamped to the last 16-byte granule holding content
// (a no-op except in a chunk's partial last step): addresses stay inside the
// chunk's pages and every call is one straight-line path of exactly 4 loads,
// so the compiler's vmcnt bookkeeping stays exact across the ring.
__device__ __forceinline__ void load_step(StepRegs &r, const uint8_t *cbase, uint64_t jj,
                                          uint64_t vlen, uint32_t lane)
{
    const uint64_t b0 = jj * kStep + (uint64_t) lane * kGran;
    const uint64_t last = (vlen - 1) & ~15ull;
#pragma unroll
    for (int q = 0; q < kSub; ++q) {
#if CIO_ABLATE_LOADS
        // Diagnostic build only: compute without HBM (wrong CRCs).
        const uint64_t a = min(b0 + (uint64_t) q * kRow, last) + (uint64_t) (uintptr_t) cbase;
        r.q[q] = make_uint4((uint32_t) a, (uint32_t) (a >> 7) * 0x9E3779B9u, (uint32_t) a ^ 0x5bd1e995u,
                            (uint32_t) (a >> 3) + 0x7f4a7c15u);
#else
        r.q[q] = ldg16(cbase + min(b0 + (uint64_t) q * kRow, last));
#endif
    }
}

// L64 layout (issue-ahead kernel only): lane L = 16 g + i owns the 64
// contiguous bytes [64 L, 64 L + 64) of a step, one chain per lane.  Each of
// the 4 loads still reads one whole 1 KiB row (fully coalesced): row r's
// instruction gives lane (g, i) the block 4 i + g of row r.  As a 4 x 4
// matrix of 16-lane blocks (register r, lane group g) the rows then sit
// transposed; two butterfly stages of in-register swaps -- permlane16_swap
// (groups g ^ 1 between registers r, r ^ 1) and permlane32_swap (groups g ^ 2
// between registers r, r ^ 2) -- give every owner lane its 4 blocks in
// order: register k = bytes 64 L + 16 k.  16 swaps per step replace the 3
// extra 4-lookup shifts of the 4-sub-chain layout (68 LDS lookups per step
// instead of 80) and the piece-end Horner fold.
__device__ __forceinline__ void load_step64(StepRegs &r, const uint8_t *cbase, uint64_t jj, uint32_t lane)
{
    const uint64_t b0 = jj * kStep + (uint64_t) (64u * (lane & 15u) + 16u * (lane >> 4));
#pragma unroll
    for (int q = 0; q < kSub; ++q) {
        r.q[q] = ldg16(cbase + b0 + (uint64_t) q * kRow);
    }
}

// The same with each granule clamped to the chunk's last one (general
// batches: partial last steps, as load_step).
__device__ __forceinline__ void load_step64c(StepRegs &r, const uint8_t *cbase, uint64_t jj, uint64_t vlen,
                                             uint32_t lane)
{
    const uint64_t b0 = jj * kStep + (uint64_t) (64u * (lane & 15u) + 16u * (lane >> 4));
    const uint64_t last = (vlen - 1) & ~15ull;
#pragma unroll
    for (int q = 0; q < kSub; ++q) {
        r.q[q] = ldg16(cbase + min(b0 + (uint64_t) q * kRow, last));
    }
}

__device__ __forceinline__ void swap16(uint32_t &a, uint32_t &b)
{
    const auto t = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    a = t[0];
    b = t[1];
}

__device__ __forceinline__ void swap32(uint32_t &a, uint32_t &b)
{
    const auto t = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    a = t[0];
    b = t[1];
}

__device__ __forceinline__ void transpose64(StepRegs &r)
{
    swap16(r.q[0].x, r.q[1].x); swap16(r.q[0].y, r.q[1].y); swap16(r.q[0].z, r.q[1].z); swap16(r.q[0].w, r.q[1].w);
    swap16(r.q[2].x, r.q[3].x); swap16(r.q[2].y, r.q[3].y); swap16(r.q[2].z, r.q[3].z); swap16(r.q[2].w, r.q[3].w);
    swap32(r.q[0].x, r.q[2].x); swap32(r.q[0].y, r.q[2].y); swap32(r.q[0].z, r.q[2].z); swap32(r.q[0].w, r.q[2].w);
    swap32(r.q[1].x, r.q[3].x); swap32(r.q[1].y, r.q[3].y); swap32(r.q[1].z, r.q[3].z); swap32(r.q[1].w, r.q[3].w);
}

// Generic step: partial blocks at a chunk end, and the first step of a chunk
// (alignment-head zeroing + seed fold into content bytes 0..3, which can
// straddle lanes 0 and 1 of sub-chain 0).
__device__ __forceinline__ void slow_compute(const char *lds, uint32_t lb_lo, uint32_t lb_hi,
                                             uint32_t lrep, const StepRegs &r, uint64_t jj,
                                             uint64_t vlen, uint32_t h, uint32_t seed, uint32_t lane,
                                             uint32_t (&s)[kSub], uint64_t (&e)[kSub])
{
#pragma unroll
    for (int q = 0; q < kSub; ++q) {
        const uint64_t bs = jj * kStep + (uint64_t) q * kRow + (uint64_t) lane * kGran;
        const uint32_t vb = bs >= vlen ? 0u : (uint32_t) min(vlen - bs, (uint64_t) kGran);
        if (vb == 0) {
            continue;
        }
        uint32_t w[4] = {r.q[q].x, r.q[q].y, r.q[q].z, r.q[q].w};
        if (q == 0 && jj == 0 && 16 * lane < h + 4) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int off = (int) (16 * lane) + 4 * i - (int) h;
                if (off <= -4) {
                    w[i] = 0u;
                } else if (off < 0) {
                    w[i] = (w[i] & (~0u << (8 * -off))) ^ (seed << (8 * -off));
                } else if (off == 0) {
                    w[i] ^= seed;
                } else if (off < 4) {
                    w[i] ^= seed >> (8 * off);
                }
            }
        }
        uint32_t st = step_shift(lds, lrep, s[q]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if ((uint32_t) (4 * i + 4) <= vb) {
                st = word_step(lds, lb_lo, lb_hi, st, w[i]);
            } else if ((uint32_t) (4 * i) < vb) {
                for (uint32_t t = 4 * i; t < vb; ++t) {
                    st = byte_step(lds, lb_lo, st, (w[i] >> (8 * (t - 4 * i))) & 0xffu);
                }
            }
        }
        s[q] = st;
        e[q] = bs + vb;
    }
}

// slow_compute for the L64 layout (registers already transposed): the
// lane's one chain over its granules [64 L + 16 k, +16) of step jj, each
// clipped to the virtual length, with the head fix-up on granules 0 and 1
// of lane 0 in the chunk's first step.  A lane with no byte left in the
// step keeps its state and end.
__device__ __forceinline__ void slow_compute64(const char *lds, uint32_t lb_lo, uint32_t lb_hi, uint32_t lrep,
                                               const StepRegs &r, uint64_t jj, uint64_t vlen, uint32_t h,
                                               uint32_t seed, uint32_t lane, uint32_t &s0, uint64_t &e0)
{
    const uint64_t b0 = jj * kStep + 64ull * lane;
    if (b0 >= vlen) {
        return;
    }
    uint32_t st = step_shift(lds, lrep, s0);
#pragma unroll
    for (int k = 0; k < kSub; ++k) {
        const uint64_t bs = b0 + 16ull * (uint64_t) k;
        const uint32_t vb = bs >= vlen ? 0u : (uint32_t) min(vlen - bs, (uint64_t) kGran);
        if (vb == 0) {
            continue;
        }
        uint32_t w[4] = {r.q[k].x, r.q[k].y, r.q[k].z, r.q[k].w};
        if (jj == 0 && 64 * lane + 16 * (uint32_t) k < h + 4) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int off = 16 * k + 4 * i - (int) h;
                if (off <= -4) {
                    w[i] = 0u;
                } else if (off < 0) {
                    w[i] = (w[i] & (~0u << (8 * -off))) ^ (seed << (8 * -off));
                } else if (off == 0) {
                    w[i] ^= seed;
                } else if (off < 4) {
                    w[i] ^= seed >> (8 * off);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if ((uint32_t) (4 * i + 4) <= vb) {
                st = word_step(lds, lb_lo, lb_hi, st, w[i]);
            } else if ((uint32_t) (4 * i) < vb) {
                for (uint32_t t = 4 * i; t < vb; ++t) {
                    st = byte_step(lds, lb_lo, st, (w[i] >> (8 * (t - 4 * i))) & 0xffu);
                }
            }
        }
        e0 = bs + vb;
    }
    s0 = st;
}

// First step of a chunk on the fast path: zero the h alignment-head bytes
// and fold the seed into content bytes 0..3 (which may straddle lanes 0 and
// 1 of sub-chain 0), branch-free.  Same bytes as slow_compute's fix-up.
__device__ __forceinline__ uint4 head_fix(uint4 v, uint32_t lane, uint32_t h, uint32_t seed)
{
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int off = (int) (16 * lane) + 4 * i - (int) h;
        const uint32_t neg = (uint32_t) (-off) & 3u, pos = (uint32_t) off & 3u;
        const uint32_t keep = off <= -4 ? 0u : (off < 0 ? ~0u << (8 * neg) : ~0u);
        const uint32_t sx = (off <= -4 || off >= 4) ? 0u
                          : (off < 0 ? seed << (8 * neg) : seed >> (8 * pos));
        w[i] = (w[i] & keep) ^ sx;
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// XOR over the 64 lanes of a wave (every lane active), wave-uniform result.
// DPP moves inside each 16-lane row (quad swaps, then the half-row and row
// mirrors) leave every lane holding its row's XOR; four lane reads combine
// the rows.  Plain VALU: __shfl_xor would be six ds_bpermute round trips
// through the LDS pipe that the CRC lookups are using.
__device__ __forceinline__ uint32_t wave_xor(uint32_t v)
{
    v ^= (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
    v ^= (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
    v ^= (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x141, 0xF, 0xF, false);   // row_half_mirror
    v ^= (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x140, 0xF, 0xF, false);   // row_mirror
    return (uint32_t) (__builtin_amdgcn_readlane((int) v, 0) ^ __builtin_amdgcn_readlane((int) v, 16) ^
                       __builtin_amdgcn_readlane((int) v, 32) ^ __builtin_amdgcn_readlane((int) v, 48));
}

// A relaxed load at workgroup scope: a VECTOR load even for a uniform
// address (an outstanding scalar load would force lgkmcnt(0) on every LDS
// lookup of the CRC), counted in vmcnt with the ring's data loads.
__device__ __forceinline__ uint32_t load_vec_u32(const uint32_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// *p as a per-lane (VGPR) value: the index is an opaque zero, so the compiler
// cannot treat the load as uniform and read its result into an SGPR at once.
__device__ __forceinline__ uint32_t load_lane_u32(const uint32_t *p)
{
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return p[z];
}

// x ^ (m & c) as one v_bitop3_b32 (truth table 0x78 over x, m, c).
__device__ __forceinline__ uint32_t xor_and(uint32_t x, uint32_t m, uint32_t c)
{
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x78" : "=v"(r) : "v"(x), "v"(m), "v"(c));
    return r;
}

// All pieces of chunk c folded into one raw CRC by the last wave to publish
// one: every partial is already shifted to the chunk end (a non-final piece
// by its wave's factor F, the final piece needs none), so the fold is one
// round of independent loads and an XOR, lanes in parallel.
__device__ __forceinline__ void fold_chunk(uint32_t w0, uint32_t w1, uint32_t c, uint32_t oc,
                                           uint32_t lane, const unsigned long long *partials,
                                           const uint32_t *pfac, uint32_t *out, uint32_t *counters)
{
    // Waves w0..w1 (the plan's) hold the pieces; a wave with an empty range
    // in between has fold factor 0 in its slot, and its stale slot is skipped.
    uint32_t acc = 0;
    for (uint32_t wb = w0; wb <= w1; wb += kWave) {
        const uint32_t wv = wb + lane;
        if (wv <= w1) {
            const uint32_t p = (uint32_t) __hip_atomic_load(&partials[wv + c], __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
            acc ^= pfac[wv + c] ? p : 0u;
        }
    }
    acc = wave_xor(acc);
    if (lane == 0) {
        out[oc] = acc;
        __hip_atomic_store(&counters[c], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Tiny chunks (len < 4) and empty chunks: byte-serial with the seed, one
// chunk per lane.
__device__ __forceinline__ void tiny_chunks(const char *lds, uint32_t lb_lo, const uint8_t *base,
                                            const ChunkDesc *desc, const uint32_t *tiny,
                                            const uint32_t *seeds, uint32_t *out, const uint32_t *cid,
                                            uint32_t ntiny, uint32_t wave, uint32_t lane, uint32_t W)
{
    for (uint64_t t = (uint64_t) wave * kWave + lane; t < ntiny; t += (uint64_t) W * kWave) {
        const uint32_t c = tiny[t];
        const ChunkDesc d = desc[c];
        const uint32_t oc = cid ? cid[c] : c;
        uint32_t st = seeds ? seeds[oc] : 0xffffffffu;
        const uint8_t *p = base + d.a + d.h;
        const uint32_t len = (uint32_t) (d.vlen - d.h);
        for (uint32_t i = 0; i < len; ++i) {
            st = byte_step(lds, lb_lo, st, p[i]);
        }
        out[oc] = st;
    }
}

// The CRC kernel: one launch per batch.
//   1. every workgroup builds the LDS tables (160 KiB);
//   2. every wave streams its even share of the batch's wave-steps through a
//      D-deep register ring (loads for step g+D issued while step g is CRC'd),
//      publishing one partial CRC per chunk piece;
//   3. the last wave to publish a piece of a chunk folds the chunk;
//   4. chunks shorter than 4 bytes are done byte-serially.
// Rotate this wave's issue priority so that, over any 4 consecutive ring
// iterations, every wave of a SIMD holds each priority level once: the
// hardware's age tie-break otherwise lets the oldest wave of each SIMD run
// ~30% ahead of the youngest, and the workgroup ends with the youngest.
__device__ __forceinline__ void rotate_prio(uint32_t slot_group, uint64_t it)
{
    switch ((slot_group + (uint32_t) it) & 3u) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
    }
}

// UNIFORM: the plan's batch is uniform (equal lengths, constant stride), so
// a wave's first chunk and its descriptor follow from the kernel arguments
// alone (all preloaded into SGPRs): the first HBM requests wait on no memory
// access.  The general path reads its WaveStart record first.  Separate
// instantiations keep the general path's scalar-load wait out of the
// uniform one's prologue.
// (CIO_DIAG_NO_ARRIVAL, CIO_LDS_FOLD, CIO_DIAG_TAIL: cio_diag.h.)
// AHEAD (uniform batches of whole 4 KiB steps with no alignment head: every
// step is full, so the partial-step paths compile out): two ring slots, and
// the next step's loads are issued as soon as this step's data has landed,
// BEFORE its CRC -- still one step (4 KiB) in flight per wave, as in the
// read-only stream, but no longer none while the wave computes.
template <bool STAMPS = false, int PRIO = 1, bool UNIFORM = false, bool AHEAD = false, bool L64 = false>
__global__ void __launch_bounds__(kThreads, 1)
crc32_stream_kernel(const uint8_t *base, uint64_t S, uint64_t ustride, uint64_t ua0, uint64_t uvlen,
                    uint32_t W, uint32_t unsteps, uint32_t uh, uint32_t n,
                    const ChunkDesc *__restrict__ desc,
                    const WaveStart *__restrict__ wstart, const uint32_t *__restrict__ tiny,
                    const uint32_t *__restrict__ seeds, uint32_t *out, const uint32_t *__restrict__ cid,
                    unsigned long long *__restrict__ partials, uint32_t *__restrict__ counters,
                    const uint32_t *__restrict__ g_slice, const uint32_t *__restrict__ g_shift,
                    const uint32_t *__restrict__ g_x8, const uint32_t *__restrict__ pfac,
                    uint32_t ntiny, unsigned long long *stamps)
{
    __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
    const uint32_t tid = threadIdx.x;
    unsigned long long t_entry = 0, t_tables = 0, t_stream = 0, t_first = 0, t_mid = 0, t_issued = 0;
    unsigned long long t_wt[2] = {0, 0}, t_step1 = 0, t_arrived = 0, t_bar1 = 0, t_bar2 = 0, t_folded = 0;
    if (STAMPS) {
        t_entry = __builtin_amdgcn_s_memrealtime();
    }

    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (kThreads / kWave) + (tid >> 6));
    const uint32_t lane = tid & 63u;
    const uint32_t lb_lo = (lane & kSliceRepMask) << 2;
    const uint32_t lb_hi = lb_lo | 0x10000u;
    const uint32_t lrep = (lane & kShiftRepMask) << 2;
    const uint32_t slot_group = __builtin_amdgcn_readfirstlane((tid >> 6) >> 2);
    const uint64_t g0 = uniform_u64(wave_start(wave, S, W));
    const uint64_t gend = uniform_u64(wave_start((uint64_t) wave + 1, S, W));
    const bool active = g0 < gend;

    // Compute cursor (c, d, j) and load cursor (lc, ld, lj) walk the same
    // step sequence; the load cursor runs one step ahead.
    uint32_t c = 0, lc = 0, c0 = 0;
    ChunkDesc d = {}, ld = {};
    uint32_t j = 0, lj = 0;    // step within the chunk (nsteps is 32-bit)
    uint64_t nload = 0;
    if (active) {
        if (UNIFORM) {
            // Uniform batch (equal lengths, constant 16-byte-multiple stride):
            // the first chunk and its descriptor follow from the kernel
            // arguments, so the first loads wait on no memory access.
            // S = n * unsteps, so floor(g0 / unsteps) = floor(wave * n / W).
            c = __builtin_amdgcn_readfirstlane((uint32_t) split_point(wave, n, W));
            d.a = ua0 + (uint64_t) c * ustride;
            d.vlen = uvlen;
            d.g = (uint64_t) c * unsteps;
            d.nsteps = unsteps;
            d.h = uh;
        } else {
            const WaveStart ws = wstart[wave];
            c = ws.c;
            d = ws.d;
        }
        c0 = c;
        j = (uint32_t) (g0 - d.g);
        lc = c;
        ld = d;
        lj = j;
        nload = gend - g0;
    }

    // Waves without steps (only when the batch has fewer steps than waves)
    // point their loads at bytes that are always readable: the first granule
    // of chunk 0 in a uniform batch (every chunk there has >= 4 content
    // bytes), else the 4 KiB slice table.  The uniform choice needs no
    // kernel-argument load, so nothing in the uniform prologue waits on one.
    const uint8_t *lbase = (UNIFORM || active) ? base : reinterpret_cast<const uint8_t *>(g_slice);
    if (!active) {
        ld.a = UNIFORM ? ua0 : 0;
        ld.vlen = kGran;
        ld.nsteps = 1;
    }

    auto issue = [&](StepRegs &r) {
        // Past the wave's range the last step is re-read (cache-resident) so
        // that every refill is the same 4 loads.  AHEAD refills past the
        // range (its last one, or none when CIO_AHEAD_PEEL peels the last
        // step) use a dummy source chosen branch-free, so one load sequence
        // serves every path and the compiler's vmcnt waits stay exact: in a
        // uniform batch chunk 0's first step at base + ua0 (both preloaded
        // SGPRs -- the slice-table pointer is a kernel argument the hardware
        // does not preload, and its scalar load held every wave's first HBM
        // request), otherwise the L2-resident 4 KiB slice table.
        if (AHEAD) {
            const bool real = nload > 0;
            const uint8_t *src = real ? lbase + ld.a
                               : UNIFORM ? base + ua0 : reinterpret_cast<const uint8_t *>(g_slice);
            if (L64) {
                load_step64(r, src, real ? lj : 0, lane);
            } else {
                load_step(r, src, real ? lj : 0, real ? ld.vlen : (uint64_t) kStep, lane);
            }
        } else {
        const uint64_t jj = nload > 0 ? lj : (uint64_t) ld.nsteps - 1;
        if (L64) {
            load_step64c(r, lbase + ld.a, jj, ld.vlen, lane);
        } else {
            load_step(r, lbase + ld.a, jj, ld.vlen, lane);
        }
        }
        if (nload > 0) {
            --nload;
            if (++lj == ld.nsteps && nload > 0) {
                if (UNIFORM) {
                    ++lc;
                    ld.a += ustride;
                    ld.g += unsteps;
                } else {
                    do {
                        ++lc;
                        ld = desc[lc];
                    } while (ld.nsteps == 0);
                }
                lj = 0;
            }
        }
    };

    // Table entries are computed, not loaded: at kernel start every global
    // load pays cold-cache latency, and the build sits on the critical path.
    auto build_tables = [&]() {
        uint32_t tab_v[kE], tab_sv[kE];
#pragma unroll
        for (int e = 0; e < kE; ++e) {
            const uint32_t idx = tid + (uint32_t) kThreads * e;
            table_entries<L64 ? cx_xpow8n(kStep - 64) : kXStepShift>(__builtin_amdgcn_readfirstlane(idx >> 8),
                                                                     idx & 255u, tab_v[e], tab_sv[e]);
        }
        write_tables<STAMPS>(lds, tid, tab_v, tab_sv, t_wt);
    };
    // The first step is requested before the table build so that its HBM
    // latency overlaps it (requesting two was slower: profiles/r01/ab_v4_steps.txt).
    // Unconditional (also for inactive waves): a branch here would merge a
    // no-load path into the vmcnt state and make the table build wait for the ring.
    StepRegs cur, nxt;
    issue(cur);
    // The data requests leave first; the bookkeeping loads below need
    // kernel-argument pointers (scalar loads) and must not hold them back.
    __builtin_amdgcn_sched_barrier(0);
    // Descriptors of the first 64 chunks from c0 (one per lane) for the
    // arrival step at the end; fetched now so that they cost nothing there.
    // Clamped, not predicated: a branch would break the ring's vmcnt tracking.
    uint64_t ar_g = 0;
    uint32_t ar_ns = 0, ar_np = 0, ar_w0 = 0, ar_w1 = 0;
    if (CIO_DIAG_NO_ARRIVAL < 2) {
        const ChunkDesc &ad = desc[min(c0 + lane, n - 1)];
        ar_g = ad.g;
        ar_ns = ad.nsteps;
        ar_np = ad.npieces;
        ar_w0 = ad.w0;
        ar_w1 = ad.w1;
    }
    // Fold factor of a piece that ends with a full step (the common case):
    // sub-chain q of lane l then ends 1024 (3 - q) + 16 (63 - l) bytes before
    // the piece end.  The 1024 (3 - q) parts are compile-time constants
    // (fold_full); the lane part x^(8 * 16 (63 - l)) is fetched once here
    // instead of gathered from g_x8 at every piece end.
    const uint32_t xl = g_x8[L64 ? 64u * (63u - lane) : kRow - (lane + 1) * kGran];
    // Workgroup-local fold.  A split chunk whose pieces all lie in this
    // workgroup's 16 waves skips the partial slot and the arrival counter:
    // each non-final piece (a wave's last piece) goes to the wave's LDS word
    // once the stream is over, and the wave holding the final piece (its
    // first chunk c0, begun before its range) folds them there.  Its fold
    // factors are fetched now, so the fold at the end waits on no HBM access.
    // The plan's per-wave words follow the piece slots: the LDS-fold flags
    // (kWfFold, kWfPublish) and the fold factor of the wave's last piece
    // (x^(8 * chunk bytes after it); 1 when that piece ends its chunk).
    // Loaded as per-lane values: a uniform load's result would be moved to an
    // SGPR right here, and that wait (vmcnt, in order) would hold the table
    // build until the first step's data had landed.
    const uint32_t *wwords = pfac + (W + n + 1);
    const uint32_t wfl = CIO_LDS_FOLD ? load_lane_u32(wwords + wave) : 0u;
    const uint32_t wlast = load_lane_u32(wwords + W + wave);
    uint32_t fold_own = 0, pub = 0;
    // Keep the scheduler from sinking these loads below the table build (and
    // the table arithmetic from rising above them: the first step's HBM
    // requests leave before any table work).
    __builtin_amdgcn_sched_barrier(0);
    if (STAMPS) {
        t_issued = __builtin_amdgcn_s_memrealtime();
    }

    build_tables();
    __syncthreads();
    if (STAMPS) {
        t_tables = __builtin_amdgcn_s_memrealtime();
    }

    if (active) {
        uint32_t s[kSub] = {0u, 0u, 0u, 0u};
        uint64_t e[kSub] = {0ull, 0ull, 0ull, 0ull};
        uint32_t xlast = 0;    // F, below
        uint32_t full_end = (uint32_t) (d.vlen / kStep);
        uint32_t seed = (j == 0) ? (seeds ? seeds[cid ? cid[c] : c] : 0xffffffffu) : 0u;
        uint64_t g = g0;

        // One step: CRC the ring slot.  Returns true at a piece end (chunk or
        // range end); the piece is published by piece_end() after the next
        // step's loads are issued, so their latency overlaps the fold.
        auto crc_step = [&](StepRegs &r) -> bool {
            {
                if (L64 && (AHEAD || j < full_end)) {
                    // one chain per lane: jump 4032 bytes, then 64 contiguous bytes
                    const uint32_t h0 = step_shift(lds, lrep, s[0]);
                    transpose64(r);
                    if (j == 0) {
                        if (AHEAD) {
                            r.q[0].x ^= lane == 0 ? seed : 0u;   // h = 0: the seed on content bytes 0..3
                        } else {
                            // head bytes and seed: granules 0 and 1 of lane 0 (4 L + k);
                            // with 128-byte heads, granules 0..8 (lanes 0..2)
                            r.q[0] = head_fix(r.q[0], 4u * lane, d.h, seed);
                            r.q[1] = head_fix(r.q[1], 4u * lane + 1u, d.h, seed);
                            if (CIO_HEAD_ALIGN > 16) {
                                r.q[2] = head_fix(r.q[2], 4u * lane + 2u, d.h, seed);
                                r.q[3] = head_fix(r.q[3], 4u * lane + 3u, d.h, seed);
                            }
                        }
                    }
                    uint32_t st = block16(lds, lb_lo, lb_hi, h0, r.q[0]);
#pragma unroll
                    for (int q = 1; q < kSub; ++q) {
                        st = block16(lds, lb_lo, lb_hi, st, r.q[q]);
                    }
                    s[0] = st;
                    if (!AHEAD) {
                        e[0] = (uint64_t) j * kStep + 64ull * (lane + 1);
                    }
                } else if (L64) {
                    transpose64(r);
                    slow_compute64(lds, lb_lo, lb_hi, lrep, r, j, d.vlen, d.h, seed, lane, s[0], e[0]);
                } else if (AHEAD || j < full_end) {
                    // The 4080-byte jump of every sub-chain needs only its
                    // state: its lookups go out before the first use of the
                    // step's data, so after the data lands only the four
                    // rounds of the 16-byte update remain.
                    uint32_t h[kSub];
#pragma unroll
                    for (int q = 0; q < kSub; ++q) {
                        h[q] = step_shift(lds, lrep, s[q]);
                    }
                    if (j == 0) {
                        r.q[0] = head_fix(r.q[0], lane, d.h, seed);
                    }
#pragma unroll
                    for (int q = 0; q < kSub; ++q) {
                        s[q] = block16(lds, lb_lo, lb_hi, h[q], r.q[q]);
                    }
                    if (!AHEAD) {
                        const uint64_t e0 = (uint64_t) j * kStep + (uint64_t) (lane + 1) * kGran;
#pragma unroll
                        for (int q = 0; q < kSub; ++q) {
                            e[q] = e0 + (uint64_t) q * kRow;
                        }
                    }
                } else {
                    slow_compute(lds, lb_lo, lb_hi, lrep, r, j, d.vlen, d.h, seed, lane, s, e);
                }
                ++g;
                ++j;
                return j == d.nsteps || g == gend;
            }
        };
        // Piece end: shift every sub-chain state to the piece end, reduce over
        // the wave, publish (write-through, agent scope), move to the next chunk.
        auto piece_end = [&]() {
            {
                {
                    uint32_t contrib;
                    if (AHEAD || j <= full_end) {
                        // The last step was full: Horner over the sub-chains
                        // with the constant x^(8 * 1024), then the lane factor.
                        // (The asm keeps the compiler from hoisting xl's 32
                        // bit masks out of the loop into 64 spilled SGPRs.)
                        // A non-final piece (the range's last) takes F instead
                        // of the lane factor, landing at the chunk end.
                        uint32_t a = j < d.nsteps ? xlast : xl;
                        asm volatile("" : "+v"(a));
                        contrib = multmodp(a, L64 ? s[0] : fold_full<UNIFORM>(s));
                    } else {
                        const uint64_t pend = min((uint64_t) j * kStep, d.vlen);
                        contrib = 0;
#pragma unroll
                        for (int q = 0; q < kSub; ++q) {
                            const uint64_t dist = e[q] < pend ? pend - e[q] : 0;
                            contrib ^= s[q] ? multmodp(g_x8[min(dist, (uint64_t) (kX8Count - 1))], s[q]) : 0u;
                        }
                    }
                    contrib = wave_xor(contrib);
                    if (d.g >= g0 && j == d.nsteps) {
                        // The whole chunk lies in this wave's range: the piece
                        // is the chunk's CRC (no partial slot, no arrival).
                        if (lane == 0) {
                            out[cid ? cid[c] : c] = contrib;
                        }
                    } else if (j == d.nsteps && (wfl & kWfFold)) {
                        fold_own = contrib;    // the final piece of c0 (== c)
                    } else if (j < d.nsteps && (wfl & kWfPublish)) {
                        pub = contrib;         // the range ends inside a local chunk
                    } else {
                        __hip_atomic_store(&partials[(uint64_t) wave + c], (unsigned long long) contrib,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    if (g < gend) {
                        if (UNIFORM) {
                            ++c;
                            d.a += ustride;
                            d.g += unsteps;
                        } else {
                            do {
                                ++c;
                                d = desc[c];
                            } while (d.nsteps == 0);
                        }
                        j = 0;
#pragma unroll
                        for (int q = 0; q < kSub; ++q) {
                            s[q] = 0u;
                            e[q] = 0ull;
                        }
                        full_end = (uint32_t) (d.vlen / kStep);
                        seed = seeds ? seeds[cid ? cid[c] : c] : 0xffffffffu;
                    }
                }
            }
        };

        // One step in flight per wave (deeper rings measured slower:
        // profiles/r01/sweep_ring.txt).  Nothing is requested past the range,
        // so the wave's last CRC is not followed by a wasted round trip.
        if (STAMPS) {
            t_first = __builtin_amdgcn_s_memrealtime();
        }
        const uint64_t iters = gend - g0;
        // F = x^(8 * 16 (63 - l)) * wlast, the full fold factor of the last
        // piece per lane, so that a non-final piece lands in its slot already
        // shifted to the chunk end and no fold multiplies.  Computed in the
        // second iteration (the first if there is one), off the start-up path.
        const uint64_t it_f = iters > 1 ? 1 : 0;
        if (AHEAD) {
            // Two fixed register slots, the loop unrolled by two so each
            // slot stays one register set.  The refill of the other slot
            // goes out before this slot's CRC: the compiler's wait for this
            // slot is then vmcnt(4) (the refill's four loads may stay in
            // flight), and the wave keeps 4 KiB in flight while it computes.
            // The slot's data must have landed before the refill goes out
            // (else both slots are in flight, 8 KiB per wave, which measured
            // slower): an empty asm reading the 16 data registers makes the
            // compiler wait for them here.
            auto landed = [](StepRegs &r) {
                asm volatile("" : "+v"(r.q[0].x), "+v"(r.q[0].y), "+v"(r.q[0].z), "+v"(r.q[0].w),
                                  "+v"(r.q[1].x), "+v"(r.q[1].y), "+v"(r.q[1].z), "+v"(r.q[1].w),
                                  "+v"(r.q[2].x), "+v"(r.q[2].y), "+v"(r.q[2].z), "+v"(r.q[2].w),
                                  "+v"(r.q[3].x), "+v"(r.q[3].y), "+v"(r.q[3].z), "+v"(r.q[3].w));
            };
            auto half = [&](uint64_t it, StepRegs &use, StepRegs &fill, auto refill) {
                if (PRIO) {
                    rotate_prio(slot_group, it);
                }
                if (it == it_f) {
                    uint32_t wl = wlast;
                    asm volatile("" : "+v"(wl));
                    xlast = multmodp(wl, xl);
                }
                landed(use);
                if (decltype(refill)::value) {
                    issue(fill);    // unconditional in the loop: one load sequence on every path
                }
                if (crc_step(use)) {
                    piece_end();
                }
                if (STAMPS && it == 0) {
                    t_step1 = __builtin_amdgcn_s_memrealtime();
                }
                if (STAMPS && it == iters / 2) {
                    t_mid = __builtin_amdgcn_s_memrealtime();
                }
            };
            using Refill = std::true_type;
#if CIO_AHEAD_PEEL
            // The wave's last step is peeled off the loop: it issues no
            // refill, so the wave does not end waiting for four loads nobody
            // reads (the refill past the range re-reads the slice table; its
            // latency sat on every wave's tail, behind the vmcnt(0) below).
            using NoRefill = std::false_type;
            uint64_t it = 0;
            for (; it + 2 < iters; it += 2) {
                half(it, cur, nxt, Refill());
                half(it + 1, nxt, cur, Refill());
            }
            if (iters - it == 2) {
                half(it, cur, nxt, Refill());
                half(it + 1, nxt, cur, NoRefill());
            } else if (iters - it == 1) {
                half(it, cur, nxt, NoRefill());
            }
#else
            for (uint64_t it = 0; it < iters; it += 2) {
                half(it, cur, nxt, Refill());
                if (it + 1 < iters) {
                    half(it + 1, nxt, cur, Refill());
                }
            }
#endif
        }
        for (uint64_t it = 0; !AHEAD && it < iters; ++it) {
            if (PRIO) {
                rotate_prio(slot_group, it);
            }
            if (it == it_f) {
                // (The asm keeps the compiler from hoisting the multiply to
                // the loop's preheader, where it waited for these loads and
                // delayed every wave's first step.)
                uint32_t wl = wlast;
                asm volatile("" : "+v"(wl));
                xlast = multmodp(wl, xl);
            }
            const bool pe = crc_step(cur);
            if (STAMPS && it == 0) {
                t_step1 = __builtin_amdgcn_s_memrealtime();
            }
            if (nload > 0) {
                issue(cur);
            }
            if (pe) {
                piece_end();
            }
            if (STAMPS && it == iters / 2) {
                t_mid = __builtin_amdgcn_s_memrealtime();
            }
        }
        if (PRIO) {
            __builtin_amdgcn_s_setprio(0);
        }

        // Arrive on every chunk this wave published a piece of; the last
        // arriver folds the chunk.  The partial stores above are write-through
        // (agent scope); drain them before counting.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (STAMPS) {
            t_stream = __builtin_amdgcn_s_memrealtime();
        }
        // Lane-parallel: lane i arrives on chunk ac + i when the range holds
        // a piece of it and the chunk spans more than this range (whole
        // chunks were written out directly); the batch of 64 ends the scan
        // if it reaches a non-empty chunk that starts past the range (or the
        // end of the batch).
        for (uint32_t ac = c0; !CIO_DIAG_NO_ARRIVAL;) {
            const uint32_t idx = ac + lane;
            const bool inb = idx < n;
            const bool whole = ar_g >= g0 && ar_g + ar_ns <= gend;
            // Workgroup-local chunks (first and last piece in one workgroup)
            // were folded through LDS.
            const bool local = CIO_LDS_FOLD && (ar_w0 ^ ar_w1) < kWavesPerWg;
            const bool member = inb && ar_ns != 0 && ar_g < gend && !whole && !local;
            const bool stop = !inb || (ar_ns != 0 && ar_g >= gend);
            uint32_t old = 0;
            if (member) {
                old = __hip_atomic_fetch_add(&counters[idx], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            for (uint64_t fin = __ballot(member && old + 1 == ar_np); fin; fin &= fin - 1) {
                const uint32_t b = (uint32_t) __builtin_ctzll(fin);
                const uint32_t fc = ac + b;
                fold_chunk(__builtin_amdgcn_readlane(ar_w0, b), __builtin_amdgcn_readlane(ar_w1, b), fc,
                           cid ? cid[fc] : fc, lane, partials, pfac, out, counters);
            }
            if (__ballot(stop)) {
                break;
            }
            ac += kWave;
            const ChunkDesc &ad = desc[min(ac + lane, n - 1)];
            ar_g = ad.g;
            ar_ns = ad.nsteps;
            ar_np = ad.npieces;
            ar_w0 = ad.w0;
            ar_w1 = ad.w1;
        }
    }

    if (STAMPS) {
        t_arrived = __builtin_amdgcn_s_memrealtime();
    }
    tiny_chunks(lds, lb_lo, base, desc, tiny, seeds, out, cid, ntiny, wave, lane, W);
    if (CIO_LDS_FOLD) {
        // Every wave is past its last table lookup: the LDS words are free.
        __syncthreads();
        if (STAMPS) {
            t_bar1 = __builtin_amdgcn_s_memrealtime();
        }
        uint32_t *slot = reinterpret_cast<uint32_t *>(lds);
        if (lane == 0) {
            slot[tid >> 6] = pub;    // 0 unless the range ended inside a local chunk
        }
        __syncthreads();
        if (STAMPS) {
            t_bar2 = __builtin_amdgcn_s_memrealtime();
        }
        if (wfl & kWfFold) {
            // Lane i < 16 <-> wave (wave - 16 + i); the nb waves before this
            // one hold the chunk's earlier pieces (empty ranges published 0).
            const uint32_t nb = (wfl >> 8) & 0xffu;
            uint32_t a = 0;
            if (lane < kWavesPerWg && lane >= kWavesPerWg - nb) {
                a = slot[(tid >> 6) + lane - kWavesPerWg];
            }
            a = wave_xor(a) ^ fold_own;
            if (lane == 0) {
                out[cid ? cid[c0] : c0] = a;
            }
        }
        if (STAMPS) {
            t_folded = __builtin_amdgcn_s_memrealtime();
        }
    }
#if CIO_DIAG_TAIL == 1
    {   // diagnostic: finished waves stay resident ~5 us (sleeping) before exiting
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < 500) {
            __builtin_amdgcn_s_sleep(10);
        }
    }
#elif CIO_DIAG_TAIL == 2
    __syncthreads();   // diagnostic: finished waves wait for the workgroup before exiting
#endif
    if (STAMPS && lane == 0) {
        // Diagnostic build only: 100 MHz global clock, per wave.
        uint32_t hw_id, xcc_id;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_id));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_id));
        stamps[kStampWords * wave + 0] = t_entry;
        stamps[kStampWords * wave + 1] = t_tables;
        stamps[kStampWords * wave + 2] = t_stream;
        stamps[kStampWords * wave + 3] = __builtin_amdgcn_s_memrealtime();
        stamps[kStampWords * wave + 4] = hw_id;    // wave/simd/cu/se placement
        stamps[kStampWords * wave + 5] = xcc_id;
        stamps[kStampWords * wave + 6] = t_first;
        stamps[kStampWords * wave + 7] = t_mid;
        stamps[kStampWords * wave + 8] = t_issued;   // first step's loads issued
        stamps[kStampWords * wave + 9] = t_wt[0];    // table build: compact arrays written
        stamps[kStampWords * wave + 10] = t_wt[1];   // table build: gathered
        stamps[kStampWords * wave + 11] = t_step1;  // first step CRC'd
        stamps[kStampWords * wave + 12] = t_arrived;  // after the arrival step
        stamps[kStampWords * wave + 13] = t_bar1;     // LDS fold: past the first barrier
        stamps[kStampWords * wave + 14] = t_bar2;     // LDS fold: past the second barrier
        stamps[kStampWords * wave + 15] = t_folded;   // LDS fold done (output stored)
    }
}

// ---------------------------------------------------------------- small chunks

// Batches whose chunks all fit one wave-step (virtual length <= 4096 B, e.g.
// 4 KiB records).  Every chunk is then its own piece, so the per-chunk fold
// is what costs: the stream kernel keeps 4 independent sub-chains per lane
// (1 KiB apart) and pays a Horner pass plus a lane multiply per chunk.  Here
// the loads are the same coalesced rows (lane l gets bytes 1024 q + 16 l,
// q = 0..3), but each lane runs ONE chain through its four 16-byte blocks,
// jumping the 1008 bytes between them with the LDS shift table (built for
// 1008 instead of 4080).  The chain ends 16 (63 - l) bytes before the chunk
// end, so the fold is one multiply by x^(8 * 16 (63 - l)) -- a 32 x 32 GF(2)
// matrix held in registers, 32 masked XORs -- and a wave XOR.
//
// A chunk of virtual length v < 4096 is zero-padded to 4096 in registers:
// the padded CRC is crc * x^(8 (4096 - v)), un-shifted once per chunk by
// x^(-8 (4096 - v)) (table g_xinv8).  No partial slots, no arrival counters.
//
// Chunks are split evenly over the waves by index, output index = chunk
// index (the host pipeline's chunk-id map uses the stream kernel).  Every
// ring refill is the same loads (4 data rows; the un-shift factor unless the
// batch is uniform; the seed when seeds are given), so the compiler's vmcnt
// waits are exact.
// (CIO_SMALL_SLOTS, CIO_SMALL_EXP: cio_diag.h.)
struct SmallRegs {
    uint4 q[kSub];
    uint32_t inv;    // x^(-8 D), D = 4096 - virtual length
    uint32_t seed;   // the chunk's seed
};


// CIO_SMALL_NIBFOLD (cio_diag.h): M_L s for the lane's matrix M_L as 8 nibble
// lookups.  Table layout in the shift-table region: word (j, nib, lane) at
// kShiftOff + j * 4096 + nib * 256 + lane * 4 = M_L (nib << 4 j), so the 32
// lanes of a half-wave read 32 different banks whatever the nibbles.
// Wave w of the workgroup writes nibble position j = w / 2, nibbles
// 8 (w & 1) .. + 8, from columns 4 j .. 4 j + 3 of its lanes' matrices.
template <int J>
__device__ __forceinline__ void nib_rows(char *lds, uint32_t lane4, const uint32_t (&col)[32], uint32_t half)
{
    const uint32_t c0 = col[4 * J], c1 = col[4 * J + 1], c2 = col[4 * J + 2];
    const uint32_t c3 = col[4 * J + 3] & (0u - half);
    char *t = lds + kShiftOff + (uint32_t) J * 4096u + half * 2048u + lane4;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t v = ((k & 1) ? c0 : 0u) ^ ((k & 2) ? c1 : 0u) ^ ((k & 4) ? c2 : 0u) ^ c3;
        *reinterpret_cast<uint32_t *>(t + (uint32_t) k * 256u) = v;
    }
}

__device__ __forceinline__ void write_nib_tables(char *lds, uint32_t tid, const uint32_t (&col)[32])
{
    const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6), lane4 = (tid & 63u) << 2, half = w & 1u;
    switch (w >> 1) {
    case 0: nib_rows<0>(lds, lane4, col, half); break;
    case 1: nib_rows<1>(lds, lane4, col, half); break;
    case 2: nib_rows<2>(lds, lane4, col, half); break;
    case 3: nib_rows<3>(lds, lane4, col, half); break;
    case 4: nib_rows<4>(lds, lane4, col, half); break;
    case 5: nib_rows<5>(lds, lane4, col, half); break;
    case 6: nib_rows<6>(lds, lane4, col, half); break;
    default: nib_rows<7>(lds, lane4, col, half); break;
    }
}

__device__ __forceinline__ uint32_t nib_fold(const char *lds, uint32_t lane4, uint32_t s)
{
    const char *t = lds + kShiftOff + lane4;
    uint32_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        v[j] = *reinterpret_cast<const uint32_t *>(t + (uint32_t) j * 4096u + ((s >> (4 * j)) & 15u) * 256u);
    }
    return xor3(xor3(v[0], v[1], v[2]), xor3(v[3], v[4], v[5]), v[6] ^ v[7]);
}

// Zero the bytes of a 16-byte block at virtual offset bs past the end v.
__device__ __forceinline__ uint4 mask_tail(uint4 v, uint32_t bs, uint32_t vlen)
{
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t b = bs + 4u * i;
        const uint32_t nb = b >= vlen ? 0u : min(vlen - b, 4u);    // valid bytes of the word
        w[i] &= nb >= 4u ? ~0u : ((1u << (8u * nb)) - 1u);
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// L64 (CIO_GPU_L64): the stream kernel's L64 layout (load_step64 /
// transpose64): lane L owns bytes [64 L, 64 L + 64) of the chunk, so its
// chain runs through 64 contiguous bytes with no jump at all (64 lookups per
// chunk instead of 76) and folds with x^(8 * 64 (63 - L)).
template <bool UNI, bool SEEDS, bool L64 = false>
__global__ void __launch_bounds__(kThreads, 1)
crc32_small_kernel(const uint8_t *base, uint64_t ustride, uint64_t ua0, uint64_t uvlen, uint32_t uh,
                   uint32_t W, uint32_t n, uint32_t ntiny, const uint32_t *__restrict__ g_x8,
                   const ChunkDesc *__restrict__ desc,
                   const uint32_t *__restrict__ tiny, const uint32_t *__restrict__ seeds, uint32_t *out,
                   const uint32_t *__restrict__ g_xinv8)
{
    // (n, ntiny and g_x8 come first: the first nine arguments are preloaded
    // into SGPRs, so neither the first data requests nor the lane factor's
    // load wait on an argument load.)
    __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
    const uint32_t tid = threadIdx.x;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (kThreads / kWave) + (tid >> 6));
    const uint32_t lane = tid & 63u;
    const uint32_t lb_lo = (lane & kSliceRepMask) << 2;
    const uint32_t lb_hi = lb_lo | 0x10000u;
    const uint32_t lrep = (lane & kShiftRepMask) << 2;
    const uint32_t c0 = __builtin_amdgcn_readfirstlane((uint32_t) split_point(wave, n, W));
    const uint32_t c1 = __builtin_amdgcn_readfirstlane((uint32_t) split_point((uint64_t) wave + 1, n, W));
    const uint32_t lbyte = lane * kGran;
    // first byte this lane loads from each 1 KiB row
    const uint32_t loff = L64 ? 64u * (lane & 15u) + 16u * (lane >> 4) : lbyte;
    // Valid dummy address for the optional seeds (the value is discarded).
    const uint32_t *const seeds_p = seeds ? seeds : g_x8;

    auto geom = [&](uint32_t c, uint64_t &a, uint32_t &vlen, uint32_t &h, bool &live) {
        if (UNI) {
            a = ua0 + (uint64_t) c * ustride;
            vlen = (uint32_t) uvlen;
            h = uh;
            // Opaque per chunk: loop-invariant lane masks derived from them
            // would otherwise be hoisted into (spilled) SGPR pairs.
            asm volatile("" : "+s"(vlen), "+s"(h));
            live = true;
        } else {
            const ChunkDesc d = desc[c];
            a = d.a;
            vlen = (uint32_t) d.vlen;
            h = d.h;
            live = d.nsteps != 0;
        }
    };
    // Refill the ring slot with chunk c (past the wave's range: the last
    // chunk's geometry and the L2-resident g_x8 table as the source).
    auto issue = [&](SmallRegs &r, uint32_t c) {
        const bool in = c < c1;
        const uint32_t cc = in ? c : max(c1, 1u) - 1u;
        uint64_t a;
        uint32_t vlen, h;
        bool live;
        geom(cc, a, vlen, h, live);
        const uint32_t last = (max(vlen, 1u) - 1u) & ~15u;
        // A uniform batch re-reads its first chunk (no kernel-argument load
        // on the way to the first request); the general one the g_x8 table.
        const uint8_t *src = in ? base + a : (UNI ? base + ua0 : reinterpret_cast<const uint8_t *>(g_x8));
#pragma unroll
        for (int q = 0; q < kSub; ++q) {
            r.q[q] = ldg16(src + min(loff + (uint32_t) q * kRow, last));
        }
        if (!UNI) {
            r.inv = load_vec_u32(g_xinv8 + ((uint32_t) kStep - min(vlen, (uint32_t) kStep)));
        }
        if (SEEDS) {
            r.seed = load_vec_u32(seeds_p + cc);
        }
    };

#if CIO_SMALL_SLOTS == 2
    SmallRegs ra, rb;
    issue(ra, c0);
    issue(rb, c0 + 1);
#else
    SmallRegs cur;
    issue(cur, c0);
#endif
    __builtin_amdgcn_sched_barrier(0);
    // x^(8 * 16 (63 - l)): the lane's fold factor (the register matrix below
    // waits for it), requested right behind the first data.
    const uint32_t xl = g_x8[L64 ? 64u * (63u - lane) : kRow - kGran * (lane + 1u)];
    // Uniform batch: one un-shift factor for every chunk.
    const uint32_t inv_u = UNI ? g_xinv8[(uint32_t) kStep - min((uint32_t) uvlen, (uint32_t) kStep)] : 0u;
    __builtin_amdgcn_sched_barrier(0);
    // Table entries after the first requests (see crc32_stream_kernel).
    uint32_t tab_v[kE], tab_sv[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) {
        const uint32_t idx = tid + (uint32_t) kThreads * e;
        table_entries<cx_xpow8n(kRow - kGran)>(__builtin_amdgcn_readfirstlane(idx >> 8), idx & 255u,
                                               tab_v[e], tab_sv[e]);
    }
    constexpr bool kNib = L64 && CIO_SMALL_NIBFOLD;
    write_tables<false, !kNib>(lds, tid, tab_v, tab_sv);
    // The multiply by xl as a 32 x 32 GF(2) matrix held in registers: column
    // j = xl * x^(31 - j) (reflected bit j).
    uint32_t col[32];
    col[31] = xl;
#pragma unroll
    for (int j = 30; j >= 0; --j) {
        col[j] = (col[j + 1] >> 1) ^ (CIOA_POLY & (0u - (col[j + 1] & 1u)));
    }
    if (kNib) {
        write_nib_tables(lds, tid, col);
    }
    // Uniform batch without seeds: the head granule's fix-up (clear the bytes
    // before the content, XOR the initial 0xffffffff in) is the same for every
    // chunk, so its per-lane masks are computed once here.
    // (L64: the head and the seed, at most bytes 0..18, lie in registers 0
    // and 1 of lane 0; register k of lane L is granule 4 L + k.)
    uint32_t hk[4] = {~0u, ~0u, ~0u, ~0u}, hs[4] = {0u, 0u, 0u, 0u};
    uint32_t hk1[4] = {~0u, ~0u, ~0u, ~0u}, hs1[4] = {0u, 0u, 0u, 0u};
    if (UNI && !SEEDS) {
        const uint32_t g0 = L64 ? 4u * lane : lane;
        const uint4 k = head_fix(make_uint4(~0u, ~0u, ~0u, ~0u), g0, uh, 0u);
        const uint4 x = head_fix(make_uint4(0u, 0u, 0u, 0u), g0, uh, 0xffffffffu);
        hk[0] = k.x; hk[1] = k.y; hk[2] = k.z; hk[3] = k.w;
        hs[0] = x.x; hs[1] = x.y; hs[2] = x.z; hs[3] = x.w;
        if (L64) {
            const uint4 k1 = head_fix(make_uint4(~0u, ~0u, ~0u, ~0u), g0 + 1u, uh, 0u);
            const uint4 x1 = head_fix(make_uint4(0u, 0u, 0u, 0u), g0 + 1u, uh, 0xffffffffu);
            hk1[0] = k1.x; hk1[1] = k1.y; hk1[2] = k1.z; hk1[3] = k1.w;
            hs1[0] = x1.x; hs1[1] = x1.y; hs1[2] = x1.z; hs1[3] = x1.w;
        }
    }
    __syncthreads();

    auto chunk = [&](SmallRegs &cur, uint32_t c) {
        uint64_t a;
        uint32_t vlen, h;
        bool live;
        geom(c < c1 ? c : max(c1, 1u) - 1u, a, vlen, h, live);
        live = live && c < c1;
        uint32_t st = 0;
        const uint32_t seed = SEEDS ? cur.seed : 0xffffffffu;
        if (live) {
            StepRegs r;
#pragma unroll
            for (int q = 0; q < kSub; ++q) {
                r.q[q] = cur.q[q];
            }
            if (L64) {
                transpose64(r);
            }
            if (UNI && !SEEDS) {
                r.q[0] = make_uint4((r.q[0].x & hk[0]) ^ hs[0], (r.q[0].y & hk[1]) ^ hs[1],
                                    (r.q[0].z & hk[2]) ^ hs[2], (r.q[0].w & hk[3]) ^ hs[3]);
                if (L64) {
                    r.q[1] = make_uint4((r.q[1].x & hk1[0]) ^ hs1[0], (r.q[1].y & hk1[1]) ^ hs1[1],
                                        (r.q[1].z & hk1[2]) ^ hs1[2], (r.q[1].w & hk1[3]) ^ hs1[3]);
                }
            } else if (L64) {
                r.q[0] = head_fix(r.q[0], 4u * lane, h, seed);
                r.q[1] = head_fix(r.q[1], 4u * lane + 1u, h, seed);
            } else {
                r.q[0] = head_fix(r.q[0], lane, h, seed);
            }
            if (vlen < (uint32_t) kStep) {
#pragma unroll
                for (int q = 0; q < kSub; ++q) {
                    r.q[q] = mask_tail(r.q[q], L64 ? 64u * lane + 16u * (uint32_t) q : lbyte + (uint32_t) q * kRow,
                                       vlen);
                }
            }
            if (CIO_SMALL_EXP & 2) {
#pragma unroll
                for (int q = 0; q < kSub; ++q) {
                    st ^= r.q[q].x ^ r.q[q].y ^ r.q[q].z ^ r.q[q].w;
                }
            } else {
                // (the chain starts at 0: its first block needs no jump)
                st = block16(lds, lb_lo, lb_hi, 0u, r.q[0]);
#pragma unroll
                for (int q = 1; q < kSub; ++q) {
                    st = L64 ? block16(lds, lb_lo, lb_hi, st, r.q[q])
                             : shift_block16(lds, lb_lo, lb_hi, lrep, st, r.q[q]);
                }
            }
        }
        uint32_t inv = inv_u;
        if (!UNI) {
            asm volatile("v_mov_b32 %0, %1" : "=v"(inv) : "v"(cur.inv));
        }
        // The next chunk's loads go out before the fold.
        issue(cur, c + CIO_SMALL_SLOTS);
        if (live) {
            uint32_t x = st;
            if (kNib && !(CIO_SMALL_EXP & 1)) {
                x = nib_fold(lds, lane << 2, st);
            } else if (!(CIO_SMALL_EXP & 1)) {
                // 32 x (bit-field sign extend, fused and-xor)
                x = col[0] & (0u - (st & 1u));
#pragma unroll
                for (int j = 1; j < 32; ++j) {
                    x = xor_and(x, 0u - ((st >> j) & 1u), col[j]);
                }
            }
            uint32_t crc = wave_xor(x);
            if (vlen != (uint32_t) kStep) {
                asm volatile("" : "+v"(inv));   // (no hoisting of inv's bit masks into SGPRs)
                crc = multmodp(inv, crc);
            }
            if (lane == 0) {
                out[c] = crc;
            }
        }
    };
#if CIO_SMALL_SLOTS == 2
    for (uint32_t c = c0; c < c1; c += 2) {
        chunk(ra, c);
        chunk(rb, c + 1);
    }
#else
    // Issue priority rotates per chunk as in the stream kernel, so no wave of
    // a SIMD stays behind its mates under the age tie-break (cfg4k 68.7 ->
    // 66.6 us back to back, profiles/r02/ab_small_prio_rotation.txt).
    const uint32_t slot_group = __builtin_amdgcn_readfirstlane((tid >> 6) >> 2);
    for (uint32_t c = c0; c < c1; ++c) {
        rotate_prio(slot_group, c - c0);   // (reversed or every-2-chunks rotation: neutral)
        chunk(cur, c);
    }
    __builtin_amdgcn_s_setprio(0);
#endif
    tiny_chunks(lds, lb_lo, base, desc, tiny, seeds, out, nullptr, ntiny, wave, lane, W);
}

// ---------------------------------------------------------------- read-only stream

// Practical HBM-read ceiling for the CRC kernel's access pattern: the same
// persistent grid (one 1024-thread workgroup per CU), the same even split of
// 4 KiB wave-steps and the same coalesced non-temporal 16-byte loads, with the
// CRC replaced by an XOR.  One 4-byte store per wave keeps the loads live.
__global__ void __launch_bounds__(kThreads, 1)
read_stream_kernel(const uint8_t *__restrict__ base, uint64_t S, uint32_t *__restrict__ sink, uint32_t B,
                   unsigned long long *stamps, uint32_t work)
{
    const unsigned long long t_entry = stamps ? __builtin_amdgcn_s_memrealtime() : 0;
    unsigned long long t_first = 0;
    const uint32_t W = gridDim.x * (kThreads / kWave);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (kThreads / kWave) + (threadIdx.x >> 6));
    const uint32_t lane = threadIdx.x & 63u;
    u32x4 acc = {0u, 0u, 0u, 0u};
    // diagnostic (CIO_GPU_RS_WORK=n): n rounds of 4 independent dependent
    // chains of full-rate VALU work (3 instructions per chain and round) on
    // each step's data, standing in for the CRC's arithmetic.
    auto burn = [&]() {
        uint32_t x0 = acc.x, x1 = acc.y, x2 = acc.z, x3 = acc.w;
        for (uint32_t k = 0; k < work; ++k) {
            x0 = __builtin_amdgcn_alignbit(x0, x0, 27) ^ (x0 + k);
            x1 = __builtin_amdgcn_alignbit(x1, x1, 27) ^ (x1 + k);
            x2 = __builtin_amdgcn_alignbit(x2, x2, 27) ^ (x2 + k);
            x3 = __builtin_amdgcn_alignbit(x3, x3, 27) ^ (x3 + k);
        }
        acc = u32x4{x0, x1, x2, x3};
    };
    // diagnostic (CIO_GPU_RS_LANE): lane l reads 32 or 64 contiguous bytes of
    // each half / whole step (2 or 4 dwordx4 loads at a 32 / 64-byte lane
    // stride) instead of 16 bytes of each 1 KiB row.
    const uint32_t lsh = work >> 16;
    work &= 0xffffu;
    auto step = [&](uint64_t g) {
        if (lsh == 0) {
            const u32x4 *p = reinterpret_cast<const u32x4 *>(base + g * kStep + (uint64_t) lane * kGran);
#pragma unroll
            for (int q = 0; q < kSub; ++q) {
                acc ^= __builtin_nontemporal_load(p + q * kWave);
            }
        } else if (lsh == 1) {
            const u32x4 *p = reinterpret_cast<const u32x4 *>(base + g * kStep + (uint64_t) lane * 32u);
            acc ^= __builtin_nontemporal_load(p);
            acc ^= __builtin_nontemporal_load(p + 1);
            acc ^= __builtin_nontemporal_load(p + 128);
            acc ^= __builtin_nontemporal_load(p + 129);
        } else {
            const u32x4 *p = reinterpret_cast<const u32x4 *>(base + g * kStep + (uint64_t) lane * 64u);
#pragma unroll
            for (int q = 0; q < kSub; ++q) {
                acc ^= __builtin_nontemporal_load(p + q);
            }
        }
        burn();
    };
    if (B == 0xffffffffu) {
        // diagnostic (CIO_GPU_RS_BLOCK=-1): the contiguous split with two
        // steps in flight per wave (the last two refills re-read the last step)
        const uint64_t g0 = wave_start(wave, S, W), g1 = wave_start((uint64_t) wave + 1, S, W);
        if (g0 < g1) {
            auto ld4 = [&](u32x4 *r, uint64_t g) {
                const u32x4 *p = reinterpret_cast<const u32x4 *>(base + min(g, g1 - 1) * kStep +
                                                                 (uint64_t) lane * kGran);
#pragma unroll
                for (int q = 0; q < kSub; ++q) {
                    r[q] = __builtin_nontemporal_load(p + q * kWave);
                }
            };
            u32x4 ra[kSub], rb[kSub];
            ld4(ra, g0);
            ld4(rb, g0 + 1);
            for (uint64_t g = g0; g < g1; g += 2) {
#pragma unroll
                for (int q = 0; q < kSub; ++q) {
                    acc ^= ra[q];
                }
                ld4(ra, g + 2);
                __builtin_amdgcn_sched_barrier(0);
                burn();
#pragma unroll
                for (int q = 0; q < kSub; ++q) {
                    acc ^= rb[q];
                }
                ld4(rb, g + 3);
                __builtin_amdgcn_sched_barrier(0);
                burn();
            }
        }
    } else if (B & 0x80000000u) {
        // diagnostic (CIO_GPU_RS_WGPOOL=k): the CRC kernel's split, but the
        // last k steps of every wave's range form a workgroup pool that the
        // workgroup's waves claim one step at a time (LDS atomic) once their
        // own ranges are done: intra-workgroup balancing, priced on the
        // read-only stream.
        __shared__ uint32_t pool_next;
        const uint32_t k = B & 0xffffu;
        if (threadIdx.x == 0) {
            pool_next = 0;
        }
        __syncthreads();
        auto static_end = [&](uint64_t w, uint64_t &e1) {
            const uint64_t a = wave_start(w, S, W), b = wave_start(w + 1, S, W);
            e1 = b;
            return b > a + k ? b - k : a;
        };
        uint64_t g1;
        const uint64_t g0 = wave_start(wave, S, W), gs = static_end(wave, g1);
        for (uint64_t g = g0; g < gs; ++g) {
            step(g);
        }
        const uint32_t first = blockIdx.x * (kThreads / kWave);
        for (;;) {
            uint32_t item = 0;
            if (lane == 0) {
                item = atomicAdd(&pool_next, 1u);
            }
            item = __builtin_amdgcn_readfirstlane(item);
            if (item >= (kThreads / kWave) * k) {
                break;
            }
            uint64_t o1;
            const uint64_t os = static_end(first + item / k, o1);
            const uint64_t g = os + item % k;
            if (g < o1) {
                step(g);
            }
        }
    } else if (B == 0) {
        // the CRC kernel's split: one contiguous range per wave
        const uint64_t g0 = wave_start(wave, S, W), g1 = wave_start((uint64_t) wave + 1, S, W);
        for (uint64_t g = g0; g < g1; ++g) {
            step(g);
            if (stamps && g == g0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                t_first = __builtin_amdgcn_s_memrealtime();
            }
        }
    } else {
        // diagnostic (CIO_GPU_RS_BLOCK=B): blocks of B steps dealt round-robin over the waves
        for (uint64_t b = wave; b * B < S; b += W) {
            for (uint64_t g = b * B; g < min(S, b * B + B); ++g) {
                step(g);
            }
        }
    }
    const uint32_t x = wave_xor(acc[0] ^ acc[1] ^ acc[2] ^ acc[3]);
    if (lane == 0) {
        sink[wave] = x;
    }
    if (stamps && lane == 0) {
        // Diagnostic (CIO_GPU_RS_STAMPS=1): 100 MHz global clock, per wave.
        uint32_t xcc_id;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_id));
        stamps[4 * wave + 0] = t_entry;
        stamps[4 * wave + 1] = t_first;
        stamps[4 * wave + 2] = __builtin_amdgcn_s_memrealtime();
        stamps[4 * wave + 3] = xcc_id;
    }
}

// ---------------------------------------------------------------- synthetic fill

__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256)
fill_kernel(uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
            const uint64_t *__restrict__ lens, const uint64_t *__restrict__ ids, uint64_t seed,
            uint32_t n)
{
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint64_t off = offs[i], len = lens[i];
        if (len == 0) {
            continue;
        }
        const uint64_t id = ids ? ids[i] : (uint64_t) i;
        const uint64_t key = seed ^ (0x9E3779B97F4A7C15ull * (id + 1));
        const uint64_t first = off & ~15ull;
        const uint64_t ngran = ((off + len + 15) & ~15ull) - first;
        for (uint64_t gi = threadIdx.x; gi < ngran / 16; gi += blockDim.x) {
            const uint64_t gaddr = first + gi * 16;
            const int64_t t0 = (int64_t) gaddr - (int64_t) off;  // chunk-relative byte of granule start
            if (t0 >= 0 && (uint64_t) t0 + 16 <= len) {
                const uint64_t k0 = (uint64_t) t0 >> 3;
                const uint32_t sh = (uint32_t) (t0 & 7) * 8;
                const uint64_t w0 = splitmix64(key + k0), w1 = splitmix64(key + k0 + 1);
                uint64_t lo, hi;
                if (sh == 0) {
                    lo = w0; hi = w1;
                } else {
                    const uint64_t w2 = splitmix64(key + k0 + 2);
                    lo = (w0 >> sh) | (w1 << (64 - sh));
                    hi = (w1 >> sh) | (w2 << (64 - sh));
                }
                *reinterpret_cast<uint4 *>(base + gaddr) =
                    make_uint4((uint32_t) lo, (uint32_t) (lo >> 32), (uint32_t) hi, (uint32_t) (hi >> 32));
            } else {
                for (int b = 0; b < 16; ++b) {
                    const int64_t t = t0 + b;
                    if (t >= 0 && (uint64_t) t < len) {
                        const uint64_t w = splitmix64(key + ((uint64_t) t >> 3));
                        base[gaddr + b] = (uint8_t) (w >> (8 * (t & 7)));
                    }
                }
            }
        }
    }
}

#if defined(CIO_DIAG_RS_DYN)
// Diagnostic (CIO_GPU_RS_DYN="pool_permille,U,NC"): the read-only stream with
// a dynamic tail.  The first S - P steps are split evenly over the waves as
// in read_stream_kernel; the last P steps form a pool of U-step units, dealt
// over NC counters (one cache line each).  A wave that has finished its
// static range claims units from the counter its workgroup's XCD and slot
// hash to, moving on to the next counter when one is exhausted, so waves on
// fast CUs take over work that slow CUs would otherwise finish late.  The
// next unit is claimed before the current one is streamed (one returning
// atomic in flight).  Counters are zeroed by the host before each launch.
__global__ void __launch_bounds__(kThreads, 1)
read_stream_dyn_kernel(const uint8_t *__restrict__ base, uint64_t S, uint64_t Sst, uint32_t U,
                       uint32_t *__restrict__ ctr, uint32_t NC, uint32_t upc, uint32_t npool,
                       uint32_t *__restrict__ sink)
{
    const uint32_t W = gridDim.x * (kThreads / kWave);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (kThreads / kWave) + (threadIdx.x >> 6));
    const uint32_t lane = threadIdx.x & 63u;
    u32x4 acc = {0u, 0u, 0u, 0u};
    auto step = [&](uint64_t g) {
        const u32x4 *p = reinterpret_cast<const u32x4 *>(base + g * kStep + (uint64_t) lane * kGran);
#pragma unroll
        for (int q = 0; q < kSub; ++q) {
            acc ^= __builtin_nontemporal_load(p + q * kWave);
        }
    };
    const uint64_t g0 = wave_start(wave, Sst, W), g1 = wave_start((uint64_t) wave + 1, Sst, W);
    for (uint64_t g = g0; g < g1; ++g) {
        step(g);
    }
    // Counter c = wave mod NC: every counter is shared by waves of every XCD
    // (so a slow XCD's share flows to the others), and a wave leaves after
    // its own counter's first failed claim (one extra atomic per wave, no
    // sequential tries over other counters).  Unit k of counter c covers
    // pool steps [(k NC + c) U, +U): the counters interleave over the pool.
    const uint32_t c = wave % NC;
    auto claim = [&]() -> uint32_t {
        uint32_t u = 0;
        if (lane == 0) {
            u = __hip_atomic_fetch_add(&ctr[c * 32u], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return __builtin_amdgcn_readfirstlane(u);
    };
    uint32_t u = claim();
    while (u < upc) {
        const uint32_t unit = u * NC + c;
        u = claim();    // the next claim in flight while this unit streams
        if (unit < npool) {
            const uint64_t a = Sst + (uint64_t) unit * U;
            const uint64_t b = min(S, a + U);
            for (uint64_t g = a; g < b; ++g) {
                step(g);
            }
        }
    }
    const uint32_t x = wave_xor(acc[0] ^ acc[1] ^ acc[2] ^ acc[3]);
    if (lane == 0) {
        sink[wave] = x;
    }
}
#endif  // CIO_DIAG_RS_DYN

// ---------------------------------------------------------------- host side

}  // namespace

namespace cioa {

thread_local std::string g_err;

int fail(const char *what, hipError_t e)
{
    char buf[512];
    if (e != hipSuccess) {
        snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
    } else {
        snprintf(buf, sizeof(buf), "%s", what);
    }
    g_err = buf;
    return CIO_ERROR;
}

}  // namespace cioa

extern "C" int cioa_fail_msg(const char *what, const char *detail)
{
    g_err = std::string(what) + (detail ? std::string(": ") + detail : std::string());
    return CIO_ERROR;
}

namespace cioa {

// One DeviceState per HIP device, allocated once and never moved: plans and
// in-flight host batches keep a pointer to it (a growing vector
// here reallocated under them when a second device was first used).
std::mutex g_mu;
std::unique_ptr<DeviceState> g_dev[kMaxDev];

int device_state(DeviceState **out)
{
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    if (dev < 0 || dev >= kMaxDev) {
        return fail("device ordinal out of range");
    }
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_dev[dev]) {
        g_dev[dev].reset(new DeviceState());
    }
    DeviceState &st = *g_dev[dev];
    if (!st.ready) {
        hipDeviceProp_t prop;
        HIP_TRY(hipGetDeviceProperties(&prop, dev), "hipGetDeviceProperties");
        if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            char msg[256];
            snprintf(msg, sizeof(msg), "chunkio_amd kernels are built for gfx950, device is %s",
                     prop.gcnArchName);
            return fail(msg);
        }
        st.cus = prop.multiProcessorCount;
        static uint32_t slice[4][256], shift[4][256];
        std::vector<uint32_t> x8(kX8Count);
        cioa_gen_slice4(slice);
        cioa_gen_shift_table(shift, (uint64_t) (kStep - kGran));
        cioa_gen_xpow8_table(x8.data(), kX8Count, 1);
        HIP_TRY(hipMalloc(&st.slice, sizeof(slice)), "hipMalloc(slice)");
        HIP_TRY(hipMalloc(&st.shift, sizeof(shift)), "hipMalloc(shift)");
        HIP_TRY(hipMalloc(&st.x8, kX8Count * sizeof(uint32_t)), "hipMalloc(x8)");
        HIP_TRY(hipMemcpy(st.slice, slice, sizeof(slice), hipMemcpyHostToDevice), "upload slice");
        HIP_TRY(hipMemcpy(st.shift, shift, sizeof(shift), hipMemcpyHostToDevice), "upload shift");
        HIP_TRY(hipMemcpy(st.x8, x8.data(), kX8Count * sizeof(uint32_t), hipMemcpyHostToDevice),
                "upload x8");
        // x^-1 = (P(x) - 1) / x, reflected: P's low coefficients moved down one power.
        std::vector<uint32_t> xinv8(kStep);
        uint32_t xm8 = 0x80000000u;
        for (int i = 0; i < 8; ++i) {
            xm8 = cioa_multmodp(xm8, (CIOA_POLY << 1) | 1u);
        }
        xinv8[0] = 0x80000000u;
        for (int d = 1; d < kStep; ++d) {
            xinv8[d] = cioa_multmodp(xinv8[d - 1], xm8);
        }
        HIP_TRY(hipMalloc(&st.xinv8, kStep * sizeof(uint32_t)), "hipMalloc(xinv8)");
        HIP_TRY(hipMemcpy(st.xinv8, xinv8.data(), kStep * sizeof(uint32_t), hipMemcpyHostToDevice),
                "upload xinv8");
        st.ready = true;
    }
    *out = &st;
    return CIO_OK;
}

}  // namespace cioa

extern "C" {

const char *cio_gpu_last_error(void)
{
    return g_err.c_str();
}

const char *cio_gpu_version(void)
{
#define CIO_STR2(x) #x
#define CIO_STR(x) CIO_STR2(x)
    return "chunkio_amd crc32 v9 gfx950 stream(l64-lanes permlane-transpose issue-ahead<=64steps pre-shift prio-rotate "
           "coalesced-nt division-free-start slice4-lds32x perm direct-whole preshifted-partials wg-lds-fold "
           "head-align=" CIO_STR(CIO_HEAD_ALIGN) ") "
           "small(4x16B dpp-reduce bitop3-fold prio-rotate) "
           "host(nt-staging graduated-groups pread-bounce multi-device vpclmul-crc_update small-batch-route) "
           "sha1(2-schedule-waves 4-block-handover continuation)";
}

int cio_gpu_init(void)
{
    DeviceState *st;
    return device_state(&st);
}

void cio_crc32_plan_destroy(cio_crc32_plan *p)
{
    if (!p) {
        return;
    }
    (void) hipFree(p->desc);
    (void) hipFree(p->wstart);
    (void) hipFree(p->tiny);
    (void) hipFree(p->partials);
    (void) hipFree(p->counters);
    (void) hipFree(p->pfac);
    (void) hipFree(p->stamps);
    delete p;
}

}  // extern "C"

namespace cioa {

// Tuning knobs (environment, read at plan creation) and grid geometry.
void plan_init(cio_crc32_plan *p, DeviceState *st, size_t n)
{
    p->st = st;
    p->n = (uint32_t) n;
    if (const char *r = cioa_diag_getenv("CIO_GPU_PRIO")) {
        const int v = atoi(r);
        p->prio = (v == 0) ? 0 : 1;
    }
    // Lane layout of the CRC kernels (profiles/r03/ab_l64_*.txt): the
    // stream kernels take one 64-byte chain per lane (L64, permlane
    // transpose: cfg2 -5 %, cfg3 -1 %, 4 MiB chunks -1 to -2.5 %); the small
    // kernel keeps the 4-sub-chain layout (L64 there: cfg4k +1 %, 64 Ki x
    // 4 KiB -3.5 %).  CIO_GPU_L64=1 / 0 forces one layout on both.
    p->l64 = true;
    p->l64_small = false;
    if (const char *r = cioa_diag_getenv("CIO_GPU_L64")) {
        p->l64 = p->l64_small = atoi(r) != 0;
    }
    p->grid = (uint32_t) st->cus;
    // Test / A/B knob: another workgroup count (fewer than CUs: e.g. a wave
    // count that is not a power of two, which takes the kernels' f64 split
    // instead of the shift; more: workgroups that queue for a CU, up to 16
    // per CU).
    if (const char *r = cioa_diag_getenv("CIO_GPU_GRID")) {
        const int v = atoi(r);
        if (v >= 1 && v <= 16 * (int) p->grid) {
            p->grid = (uint32_t) v;
        }
    }
    p->W = p->grid * (kThreads / kWave);
}

// Virtual aligned chunks, wave-step numbering, the even split of the S steps
// over W waves, each wave's first chunk, per-chunk piece counts and per-slot
// fold factors.  Host only; returns an error message or nullptr.
const char *plan_build(PlanHost &ph, const uint64_t *offs, const uint64_t *lens, size_t n, uint32_t W)
{
    ph.desc.assign(n ? n : 1, ChunkDesc{});
    ph.tiny.clear();
    uint64_t S = 0, bytes = 0;
    for (size_t i = 0; i < n; i++) {
        ChunkDesc &d = ph.desc[i];
        const uint64_t amask = lens[i] > (uint64_t) kStep ? (uint64_t) CIO_HEAD_ALIGN - 1 : 15ull;
        d.a = offs[i] & ~amask;
        d.h = (uint32_t) (offs[i] & amask);
        d.vlen = d.h + lens[i];
        d.g = S;
        const uint64_t ns = lens[i] >= 4 ? (d.vlen + kStep - 1) / kStep : 0;
        if (ns > 0xffffffffull) {
            return "cio_crc32_plan_create: chunk too large";
        }
        d.nsteps = (uint32_t) ns;
        if (ns == 0) {
            ph.tiny.push_back((uint32_t) i);
        }
        S += ns;
        bytes += lens[i];
    }
    // The kernels' start-up divisions (div_u52) need w * S < 2^52 for w <= W
    // (W <= 2^12 on a full device: 2^40 wave-steps is 4 PiB, far past any
    // device's memory).
    if (S >= (1ull << 40) || W > 65536 || (S * (uint64_t) W) >> 52) {
        return "cio_crc32_plan_create: batch too large";
    }
    ph.S = S;
    ph.bytes = bytes;

    // Fold factors x^(8 d) for d = bytes after a piece = 4096 m + r: one
    // multiply of two table entries (x8 static, x4k per plan up to the
    // longest chunk) instead of a square-and-multiply per piece.
    static const std::vector<uint32_t> x8 = [] {
        std::vector<uint32_t> t(kStep);
        cioa_gen_xpow8_table(t.data(), kStep, 1);
        return t;
    }();
    uint64_t max_steps = 0;
    for (size_t i = 0; i < n; i++) {
        max_steps = std::max<uint64_t>(max_steps, ph.desc[i].nsteps);
    }
    std::vector<uint32_t> x4k;
    if (max_steps <= (1u << 20)) {
        x4k.resize(max_steps + 1);
        cioa_gen_xpow8_table(x4k.data(), x4k.size(), (uint64_t) kStep);
    }
    auto factor = [&](uint64_t d) {
        const uint64_t m = d / kStep, r = d % kStep;
        if (m == 0) {
            return x8[r];
        }
        return m < x4k.size() ? cioa_multmodp(x4k[m], x8[r]) : cioa_xpow8n(d);
    };

    std::vector<uint32_t> wc(W, 0), wl(W, 0);
    const size_t nslots = (size_t) W + n + 1;
    ph.pfac.assign(nslots + 2 * (size_t) W, 0u);
    if (S > 0) {
        size_t c = 0;
        for (uint32_t w = 0; w < W; w++) {
            const uint64_t g0 = ((uint64_t) w * S) / W;
            const uint64_t g1 = ((uint64_t) (w + 1) * S) / W;
            while (c < n && (ph.desc[c].nsteps == 0 || ph.desc[c].g + ph.desc[c].nsteps <= g0)) {
                c++;
            }
            wc[w] = (uint32_t) std::min(c, n - 1);
            if (g0 == g1) {
                continue;
            }
            for (size_t k = c; k < n && ph.desc[k].g < g1; k++) {
                ChunkDesc &d = ph.desc[k];
                if (d.nsteps) {
                    if (d.npieces == 0) {
                        d.w0 = w;
                    }
                    d.w1 = w;
                    wl[w] = (uint32_t) k;
                    d.npieces++;
                    const uint64_t pend = std::min(std::min(g1 - d.g, (uint64_t) d.nsteps) * (uint64_t) kStep,
                                                   d.vlen);
                    ph.pfac[w + k] = factor(d.vlen - pend);
                }
            }
        }
    }
    // Workgroup-local chunks: split, with every piece in one workgroup.
    auto local = [](const ChunkDesc &d) {
        return d.npieces > 1 && d.w0 / kWavesPerWg == d.w1 / kWavesPerWg;
    };
    for (uint32_t w = 0; S > 0 && w < W; w++) {
        const uint64_t g0 = ((uint64_t) w * S) / W;
        const uint64_t g1 = ((uint64_t) (w + 1) * S) / W;
        if (g0 == g1) {
            continue;
        }
        uint32_t f = 0;
        const ChunkDesc &first = ph.desc[wc[w]];
        if (first.g < g0 && first.g + first.nsteps <= g1 && local(first)) {
            f |= kWfFold | ((w - first.w0) << 8);
        }
        const ChunkDesc &last = ph.desc[wl[w]];
        const bool nonfinal = last.g + last.nsteps > g1;
        if (nonfinal && local(last)) {
            f |= kWfPublish;
        }
        ph.pfac[nslots + w] = f;
        // The last piece's factor (x^0 = 0x80000000 when it ends its chunk).
        ph.pfac[nslots + W + w] = nonfinal ? ph.pfac[w + wl[w]] : 0x80000000u;
    }
    ph.ws.assign(W, WaveStart{});
    for (uint32_t w = 0; w < W; w++) {
        ph.ws[w].c = wc[w];
        if (n) {
            ph.ws[w].d = ph.desc[wc[w]];
        }
    }
    return nullptr;
}

}  // namespace cioa

namespace {

// Uniform batch: n equal lengths >= 4 at offsets off0 + i * stride with
// stride a multiple of 16 (every chunk has the same misalignment).  The
// kernel then derives chunk descriptors arithmetically (CIO_GPU_UNIFORM=0
// disables).
void plan_uniform(cio_crc32_plan *p, const uint64_t *offs, const uint64_t *lens, size_t n, const PlanHost &ph)
{
    p->unsteps = 0;
    if (const char *r = cioa_diag_getenv("CIO_GPU_UNIFORM")) {
        if (!atoi(r)) {
            return;
        }
    }
    if (n == 0 || lens[0] < 4 || ph.desc[0].nsteps == 0) {
        return;
    }
    const uint64_t stride = n > 1 ? offs[1] - offs[0] : 0;
    if (n > 1 && (offs[1] < offs[0] || (stride & 15) != 0)) {
        return;
    }
    for (size_t i = 1; i < n; i++) {
        if (lens[i] != lens[0] || offs[i] != offs[0] + i * stride || ph.desc[i].h != ph.desc[0].h) {
            return;
        }
    }
    p->ustride = stride;
    p->ua0 = ph.desc[0].a;
    p->uvlen = ph.desc[0].vlen;
    p->uh = ph.desc[0].h;
    p->unsteps = ph.desc[0].nsteps;
}

}  // namespace

extern "C" {

int cio_crc32_plan_create(cio_crc32_plan **out, const uint64_t *offs, const uint64_t *lens, size_t n)
{
    if (!out || (n && (!offs || !lens))) {
        return fail("cio_crc32_plan_create: null argument");
    }
    if (n >= 0xffffffffull) {
        return fail("cio_crc32_plan_create: too many chunks");
    }
    *out = nullptr;
    DeviceState *st;
    if (device_state(&st) != CIO_OK) {
        return CIO_ERROR;
    }
    cio_crc32_plan *p = new cio_crc32_plan();
    plan_init(p, st, n);
    PlanHost ph;
    if (const char *err = plan_build(ph, offs, lens, n, p->W)) {
        delete p;
        return fail(err);
    }
    plan_uniform(p, offs, lens, n, ph);
    // Long batches (>= 4 MiB per wave: cfg3's ~2400 steps per wave, cfg4's
    // 2048 at one GPU) split over 4 workgroups per CU: the extra workgroups
    // queue for a CU and start wherever one finishes, so the hardware evens
    // out the per-CU finish times (cfg3 -0.7 %, cfg4 -1.7 %; shorter ranges
    // lose: 1 MiB per wave +0.8 to +5.5 %, cfg2 +5 %:
    // profiles/r04/ab_grid_oversubscribed_r04q.txt, ab_grid_cfg4_r04x.txt).
    bool oversub = false;
    if (!cioa_diag_getenv("CIO_GPU_GRID") && ph.S >= 1024ull * p->W && 4ull * p->W <= 65536 &&
        ph.S != (uint64_t) n - ph.tiny.size()) {    // (not a small-chunk batch)
        PlanHost ph4;
        if (plan_build(ph4, offs, lens, n, 4 * p->W) == nullptr) {
            p->grid *= 4;
            p->W *= 4;
            oversub = true;
            ph = std::move(ph4);
        }
    }
    // HBM channel camping (profiles/r05/camping/): when every wave's range is
    // the same multiple of 16 steps (64 KiB), all waves read addresses equal
    // modulo 64 KiB at the same moment and even the read-only stream loses
    // 5-10 % (16, 32, 64 steps per wave against 17, 33, 65).  One workgroup
    // fewer per 32 -- one per XCD, so the XCDs stay balanced -- makes the
    // ranges uneven and breaks the congruence.  Warm ABBA A/B
    // (ab_anticamp_abba_r05x.txt): stream kernel +4.1 to +4.6 % at 16-64
    // steps per wave, -1.0 % at 128 and 256; small-chunk kernel +10.9 to
    // +14.3 % at 16-64 chunks per wave, +3.9 % at 128.  CIO_GPU_ANTICAMP=0
    // keeps the full grid; CIO_GPU_ANTICAMP_MAX overrides the range cap.
    {
        const char *r = cioa_diag_getenv("CIO_GPU_ANTICAMP");
        const bool on = !(r && atoi(r) == 0);
        const char *mx = cioa_diag_getenv("CIO_GPU_ANTICAMP_MAX");     // A/B: longest range it applies to
        const bool small_batch = ph.S > 0 && ph.S == (uint64_t) n - ph.tiny.size();
        const uint64_t wmax = mx ? strtoull(mx, nullptr, 10) : small_batch ? 128 : 64;
        const uint64_t w = p->W ? ph.S / p->W : 0;
        const bool any_grid = r && atoi(r) == 2;            // A/B: also on oversubscribed grids
        if (on && (!oversub || any_grid) && !cioa_diag_getenv("CIO_GPU_GRID") && p->grid % 32 == 0 && ph.S % p->W == 0 &&
            w % 16 == 0 &&
            w > 0 && w <= wmax) {
            const uint32_t g2 = p->grid / 32 * 31;
            PlanHost ph2;
            if (plan_build(ph2, offs, lens, n, g2 * (kThreads / kWave)) == nullptr) {
                p->grid = g2;
                p->W = g2 * (kThreads / kWave);
                ph = std::move(ph2);
            }
        }
    }
    p->S = ph.S;
    p->bytes = ph.bytes;
    p->ntiny = (uint32_t) ph.tiny.size();
    // Uniform batch of whole 4 KiB steps, 16-byte aligned, with short wave
    // ranges (<= 64 steps, e.g. cfg2's 25): the issue-ahead stream kernel.
    // Interleaved A/Bs (profiles/r03/ab_issue_ahead_*.txt): cfg2 -0.6 to
    // -1.8 %, 100- and 256-step ranges -0.3 to +0.6 % (neutral), so only
    // short ranges, where the first steps' start-up is a larger share, take
    // it.  CIO_GPU_AHEAD=1 forces it for any uniform aligned batch, 0 never.
    p->ahead = p->unsteps != 0 && p->uh == 0 && p->uvlen % kStep == 0;
    bool short_ranges = p->S <= 64ull * p->W;
    if (const char *r = cioa_diag_getenv("CIO_GPU_AHEAD")) {
        short_ranges = atoi(r) != 0;
    }
    p->ahead = p->ahead && short_ranges;

    // All chunks within one wave-step (S = number of non-tiny chunks): the
    // small-chunk kernel (CIO_GPU_SMALL=0 disables).
    p->small = ph.S > 0 && ph.S == (uint64_t) n - ph.tiny.size();
    if (const char *r = cioa_diag_getenv("CIO_GPU_SMALL")) {
        p->small = p->small && atoi(r) != 0;
    }
    if (const char *r = cioa_diag_getenv("CIO_GPU_STAMPS")) {
        if (atoi(r) > 0 && hipMalloc(&p->stamps, (size_t) p->W * kStampWords * sizeof(unsigned long long)) != hipSuccess) {
            p->stamps = nullptr;
        }
    }
    hipError_t e;
    const size_t npart = ph.pfac.size();
    if ((e = hipMalloc(&p->desc, ph.desc.size() * sizeof(ChunkDesc))) != hipSuccess ||
        (e = hipMalloc(&p->wstart, ph.ws.size() * sizeof(WaveStart))) != hipSuccess ||
        (e = hipMalloc(&p->tiny, std::max<size_t>(1, ph.tiny.size()) * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMalloc(&p->partials, npart * sizeof(unsigned long long))) != hipSuccess ||
        (e = hipMalloc(&p->counters, std::max<size_t>(1, n) * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMalloc(&p->pfac, npart * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMemcpy(p->desc, ph.desc.data(), ph.desc.size() * sizeof(ChunkDesc), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(p->wstart, ph.ws.data(), ph.ws.size() * sizeof(WaveStart), hipMemcpyHostToDevice)) != hipSuccess ||
        (ph.tiny.size() && (e = hipMemcpy(p->tiny, ph.tiny.data(), ph.tiny.size() * sizeof(uint32_t), hipMemcpyHostToDevice)) != hipSuccess) ||
        (e = hipMemset(p->partials, 0, npart * sizeof(unsigned long long))) != hipSuccess ||
        (e = hipMemset(p->counters, 0, std::max<size_t>(1, n) * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMemcpy(p->pfac, ph.pfac.data(), npart * sizeof(uint32_t), hipMemcpyHostToDevice)) != hipSuccess) {
        cio_crc32_plan_destroy(p);
        return fail("cio_crc32_plan_create: device allocation/upload", e);
    }
    *out = p;
    return CIO_OK;
}

/* A ring of `depth` plans of one geometry, each on its own stream (see the
 * header): consecutive batches overlap at their kernel edges. */
struct cio_crc32_ring {
    std::vector<cio_crc32_plan *> plans;
    std::vector<hipStream_t> streams;
    std::vector<hipEvent_t> ready, done;    // per slot: caller's inputs, slot's last batch
    std::vector<bool> pending;              // slot has work the caller has not joined
    unsigned next = 0;
    int dev = 0;                            // device the plans and streams live on
};

// Makes `dev` current for one scope and restores the caller's device after:
// a ring's plans, streams and events belong to the device current at create.
struct RingDevice {
    int prev = -1;
    hipError_t e = hipSuccess;
    explicit RingDevice(int dev)
    {
        if ((e = hipGetDevice(&prev)) == hipSuccess && prev != dev) {
            e = hipSetDevice(dev);
        }
    }
    ~RingDevice()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) {
            (void) hipSetDevice(prev);
        }
    }
};

void cio_crc32_ring_destroy(cio_crc32_ring *r)
{
    if (!r) {
        return;
    }
    RingDevice on(r->dev);
    for (hipStream_t st : r->streams) {
        if (st) (void) hipStreamSynchronize(st);
    }
    for (size_t i = 0; i < r->plans.size(); i++) {
        cio_crc32_plan_destroy(r->plans[i]);
        if (r->ready[i]) (void) hipEventDestroy(r->ready[i]);
        if (r->done[i]) (void) hipEventDestroy(r->done[i]);
        if (r->streams[i]) (void) hipStreamDestroy(r->streams[i]);
    }
    delete r;
}

int cio_crc32_ring_create(cio_crc32_ring **out, const uint64_t *offs, const uint64_t *lens, size_t n, int depth)
{
    if (!out) {
        return fail("cio_crc32_ring_create: null argument");
    }
    *out = nullptr;
    if (depth < 1 || depth > 8) {
        return fail("cio_crc32_ring_create: depth must be 1..8");
    }
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "cio_crc32_ring_create: hipGetDevice");
    cio_crc32_ring *r = new cio_crc32_ring();
    r->dev = dev;
    r->plans.assign((size_t) depth, nullptr);
    r->streams.assign((size_t) depth, nullptr);
    r->ready.assign((size_t) depth, nullptr);
    r->done.assign((size_t) depth, nullptr);
    r->pending.assign((size_t) depth, false);
    for (int i = 0; i < depth; i++) {
        if (cio_crc32_plan_create(&r->plans[(size_t) i], offs, lens, n) != CIO_OK) {
            cio_crc32_ring_destroy(r);
            return CIO_ERROR;    // (the plan's message stands)
        }
        hipError_t e = hipStreamCreateWithFlags(&r->streams[(size_t) i], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&r->ready[(size_t) i], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&r->done[(size_t) i], hipEventDisableTiming);
        if (e != hipSuccess) {
            cio_crc32_ring_destroy(r);
            return fail("cio_crc32_ring_create", e);
        }
    }
    *out = r;
    return CIO_OK;
}

int cio_crc32_ring_exec(cio_crc32_ring *r, const void *dev_base, const uint32_t *dev_seeds, uint32_t *dev_out,
                        void *stream)
{
    if (!r) {
        return fail("cio_crc32_ring_exec: null ring");
    }
    RingDevice on(r->dev);
    HIP_TRY(on.e, "cio_crc32_ring_exec: hipSetDevice");
    const size_t i = r->next % r->plans.size();
    const hipStream_t caller = reinterpret_cast<hipStream_t>(stream);
    // the batch waits for everything the caller queued before it (its inputs);
    // the slot's stream orders it after the slot's previous batch (scratch reuse)
    HIP_TRY(hipEventRecord(r->ready[i], caller), "cio_crc32_ring_exec: hipEventRecord");
    HIP_TRY(hipStreamWaitEvent(r->streams[i], r->ready[i], 0), "cio_crc32_ring_exec: hipStreamWaitEvent");
    if (plan_exec_impl(r->plans[i], dev_base, dev_seeds, dev_out, nullptr, r->streams[i]) != CIO_OK) {
        return CIO_ERROR;
    }
    HIP_TRY(hipEventRecord(r->done[i], r->streams[i]), "cio_crc32_ring_exec: hipEventRecord");
    r->pending[i] = true;
    r->next++;      // only a batch that was queued moves the ring on
    return CIO_OK;
}

int cio_crc32_ring_join(cio_crc32_ring *r, void *stream)
{
    if (!r) {
        return fail("cio_crc32_ring_join: null ring");
    }
    RingDevice on(r->dev);
    HIP_TRY(on.e, "cio_crc32_ring_join: hipSetDevice");
    const hipStream_t caller = reinterpret_cast<hipStream_t>(stream);
    for (size_t i = 0; i < r->plans.size(); i++) {
        if (r->pending[i]) {
            HIP_TRY(hipStreamWaitEvent(caller, r->done[i], 0), "cio_crc32_ring_join: hipStreamWaitEvent");
            r->pending[i] = false;
        }
    }
    return CIO_OK;
}

/* Test hook (not in the public header; host only, no device): the plan's
 * work split for W waves.  Per chunk: w0, w1, npieces (3 words); per wave:
 * the LDS-fold flags.  Returns 0, or -1 on a plan error. */
int cioa_debug_plan_layout(const uint64_t *offs, const uint64_t *lens, size_t n, uint32_t W,
                           uint32_t *chunk_words, uint32_t *wave_flags)
{
    PlanHost ph;
    if (plan_build(ph, offs, lens, n, W) != nullptr) {
        return -1;
    }
    for (size_t i = 0; i < n; i++) {
        chunk_words[3 * i + 0] = ph.desc[i].w0;
        chunk_words[3 * i + 1] = ph.desc[i].w1;
        chunk_words[3 * i + 2] = ph.desc[i].npieces;
    }
    const size_t nslots = (size_t) W + n + 1;
    for (uint32_t w = 0; w < W; w++) {
        wave_flags[w] = ph.pfac[nslots + w];
    }
    return 0;
}

/* Diagnostic (not in the public header): copy the per-wave timestamps of the
 * last launch of a CIO_GPU_STAMPS=1 plan; returns the number of waves. */
int cioa_debug_stamps(const cio_crc32_plan *p, unsigned long long *host, size_t cap)
{
    if (!p || !p->stamps) {
        return 0;
    }
    const size_t n = std::min(cap, (size_t) p->W * kStampWords);
    if (hipMemcpy(host, p->stamps, n * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) {
        return 0;
    }
    return (int) p->W;
}

uint64_t cio_crc32_plan_bytes(const cio_crc32_plan *p)
{
    return p ? p->bytes : 0;
}

uint32_t cio_crc32_plan_workgroups(const cio_crc32_plan *p)
{
    return p ? p->grid : 0;
}

const char *cio_crc32_plan_kernel(const cio_crc32_plan *p)
{
    return (p && p->small) ? "crc32_small_kernel" : "crc32_stream_kernel";
}


int cio_crc32_plan_exec_events(const cio_crc32_plan *p, const void *dev_base,
                               const uint32_t *dev_seeds, uint32_t *dev_out, void *stream,
                               void *ev_piece_start, void *ev_piece_stop)
{
    return plan_exec_impl(p, dev_base, dev_seeds, dev_out, nullptr,
                          reinterpret_cast<hipStream_t>(stream),
                          reinterpret_cast<hipEvent_t>(ev_piece_start),
                          reinterpret_cast<hipEvent_t>(ev_piece_stop));
}

int cio_crc32_plan_exec(const cio_crc32_plan *p, const void *dev_base, const uint32_t *dev_seeds,
                        uint32_t *dev_out, void *stream)
{
    return plan_exec_impl(p, dev_base, dev_seeds, dev_out, nullptr,
                          reinterpret_cast<hipStream_t>(stream));
}

}  // extern "C"

using StreamKernel = decltype(&crc32_stream_kernel<false, 1, false>);

static StreamKernel select_kernel(int prio, bool stamps, bool uniform, bool ahead, bool l64)
{
    if (ahead) {
        if (l64) {
            if (stamps) {    // per-wave stamps of the shipped cfg2 kernel (tools/stamps.py)
                return crc32_stream_kernel<true, 1, true, true, true>;
            }
            return prio ? crc32_stream_kernel<false, 1, true, true, true>
                        : crc32_stream_kernel<false, 0, true, true, true>;
        }
        return prio ? crc32_stream_kernel<false, 1, true, true> : crc32_stream_kernel<false, 0, true, true>;
    }
    if (l64 && !stamps) {
        // (uniform batches that are not aligned take the general path too: the
        // uniform L64 instantiation spilled registers)
        return prio ? crc32_stream_kernel<false, 1, false, false, true>
                    : crc32_stream_kernel<false, 0, false, false, true>;
    }
    switch ((prio ? 4 : 0) + (stamps ? 2 : 0) + (uniform ? 1 : 0)) {
    case 0: return crc32_stream_kernel<false, 0, false>;
    case 1: return crc32_stream_kernel<false, 0, true>;
    case 2: return crc32_stream_kernel<true, 0, false>;
    case 3: return crc32_stream_kernel<true, 0, true>;
    case 4: return crc32_stream_kernel<false, 1, false>;
    case 5: return crc32_stream_kernel<false, 1, true>;
    case 6: return crc32_stream_kernel<true, 1, false>;
    default: return crc32_stream_kernel<true, 1, true>;
    }
}


// One launch: stream kernel (CRC of every step, per-chunk fold by the last
// arriver, tiny chunks).  The per-chunk counters are self-resetting, so no
// memset node precedes it and the launch can be captured in a HIP graph.
int cioa::plan_exec_impl(const cio_crc32_plan *p, const void *dev_base, const uint32_t *dev_seeds,
                         uint32_t *dev_out, const uint32_t *cid, hipStream_t s,
                         hipEvent_t ev0, hipEvent_t ev1)
{
    if (!p) {
        return fail("cio_crc32_plan_exec: null plan");
    }
    if (p->n == 0) {
        return CIO_OK;
    }
    if (!dev_base || !dev_out) {
        return fail("cio_crc32_plan_exec: null buffer");
    }
    const DeviceState *st = p->st;
    if (ev0) {
        HIP_TRY(hipEventRecord(ev0, s), "hipEventRecord");
    }
    if (p->small && !cid) {
        auto sk = p->l64_small ? (p->unsteps ? (dev_seeds ? crc32_small_kernel<true, true, true>
                                                    : crc32_small_kernel<true, false, true>)
                                       : (dev_seeds ? crc32_small_kernel<false, true, true>
                                                    : crc32_small_kernel<false, false, true>))
                         : (p->unsteps ? (dev_seeds ? crc32_small_kernel<true, true> : crc32_small_kernel<true, false>)
                                       : (dev_seeds ? crc32_small_kernel<false, true>
                                                    : crc32_small_kernel<false, false>));
        hipLaunchKernelGGL(sk, dim3(p->grid), dim3(kThreads), 0, s,
                           reinterpret_cast<const uint8_t *>(dev_base), p->ustride, p->ua0, p->uvlen, p->uh,
                           p->W, p->n, p->ntiny, st->x8, p->desc, p->tiny, dev_seeds, dev_out, st->xinv8);
        HIP_TRY(hipGetLastError(), "crc32_small_kernel launch");
        if (ev1) {
            HIP_TRY(hipEventRecord(ev1, s), "hipEventRecord");
        }
        return CIO_OK;
    }
    auto kern = select_kernel(p->prio, p->stamps != nullptr, p->unsteps != 0, p->ahead && (!p->stamps || p->l64),
                              p->l64);
    hipLaunchKernelGGL(kern, dim3(p->grid), dim3(kThreads), 0, s,
                       reinterpret_cast<const uint8_t *>(dev_base), p->S, p->ustride, p->ua0, p->uvlen,
                       p->W, p->unsteps, p->uh, p->n, p->desc, p->wstart, p->tiny,
                       dev_seeds, dev_out, cid, p->partials, p->counters, st->slice, st->shift,
                       st->x8, p->pfac, p->ntiny, p->stamps);
    HIP_TRY(hipGetLastError(), "crc32_stream_kernel launch");
    if (ev1) {
        HIP_TRY(hipEventRecord(ev1, s), "hipEventRecord");
    }
    return CIO_OK;
}

extern "C" {

int cio_crc32_batch_dev(const void *dev_base, const uint64_t *offs, const uint64_t *lens,
                        const uint32_t *dev_seeds, uint32_t *dev_out, size_t n, void *stream)
{
    cio_crc32_plan *p = nullptr;
    if (cio_crc32_plan_create(&p, offs, lens, n) != CIO_OK) {
        return CIO_ERROR;
    }
    int rc = cio_crc32_plan_exec(p, dev_base, dev_seeds, dev_out, stream);
    if (rc == CIO_OK) {
        hipError_t e = hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream));
        if (e != hipSuccess) {
            rc = fail("cio_crc32_batch_dev: stream sync", e);
        }
    }
    cio_crc32_plan_destroy(p);
    return rc;
}

int cio_gpu_fill_synthetic(void *dev_base, const uint64_t *offs, const uint64_t *lens,
                           const uint64_t *ids, size_t n, uint64_t seed, void *stream)
{
    if (n == 0) {
        return CIO_OK;
    }
    DeviceState *st;
    if (device_state(&st) != CIO_OK) {
        return CIO_ERROR;
    }
    uint64_t *d_meta = nullptr;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    HIP_TRY(hipMalloc(&d_meta, 3 * n * sizeof(uint64_t)), "fill: hipMalloc");
    uint64_t *d_offs = d_meta, *d_lens = d_meta + n, *d_ids = ids ? d_meta + 2 * n : nullptr;
    hipError_t e = hipMemcpy(d_offs, offs, n * sizeof(uint64_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_lens, lens, n * sizeof(uint64_t), hipMemcpyHostToDevice);
    if (e == hipSuccess && ids) e = hipMemcpy(d_ids, ids, n * sizeof(uint64_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        const uint32_t grid = (uint32_t) std::min<size_t>(n, 65535);
        hipLaunchKernelGGL(fill_kernel, dim3(grid), dim3(256), 0, s,
                           reinterpret_cast<uint8_t *>(dev_base), d_offs, d_lens, d_ids, seed,
                           (uint32_t) n);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        e = hipStreamSynchronize(s);
    }
    (void) hipFree(d_meta);
    if (e != hipSuccess) {
        return fail("fill_kernel", e);
    }
    return CIO_OK;
}

static unsigned long long *g_rs_stamps = nullptr;   // CIO_GPU_RS_STAMPS diagnostic
static uint32_t g_rs_waves = 0;

/* Diagnostic (not in the public header): per-wave (entry, first step, done,
 * xcc) stamps of the last CIO_GPU_RS_STAMPS=1 read-stream launch; returns the
 * number of waves. */
int cioa_debug_rs_stamps(unsigned long long *host, size_t cap)
{
    if (!g_rs_stamps) {
        return 0;
    }
    const size_t n = std::min(cap, (size_t) g_rs_waves * 4);
    if (hipMemcpy(host, g_rs_stamps, n * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) {
        return 0;
    }
    return (int) g_rs_waves;
}

static int read_stream_impl(const void *dev_base, uint64_t bytes, void *stream, hipEvent_t ev0, hipEvent_t ev1,
                            uint32_t workgroups = 0);

int cio_gpu_read_stream(const void *dev_base, uint64_t bytes, void *stream)
{
    return read_stream_impl(dev_base, bytes, stream, nullptr, nullptr);
}

int cio_gpu_read_stream_grid(const void *dev_base, uint64_t bytes, uint32_t workgroups, void *stream)
{
    if (workgroups > 65536 / (kThreads / kWave)) {
        return fail("cio_gpu_read_stream_grid: more than 4096 workgroups");
    }
    return read_stream_impl(dev_base, bytes, stream, nullptr, nullptr, workgroups);
}

/* Diagnostic (not in the public header): the read-only stream with events
 * recorded right around its kernel (after the dynamic-tail counter reset). */
int cioa_debug_read_stream_events(const void *dev_base, uint64_t bytes, void *stream, void *ev0, void *ev1)
{
    return read_stream_impl(dev_base, bytes, stream, reinterpret_cast<hipEvent_t>(ev0),
                            reinterpret_cast<hipEvent_t>(ev1));
}

static int read_stream_impl(const void *dev_base, uint64_t bytes, void *stream, hipEvent_t ev0, hipEvent_t ev1,
                            uint32_t workgroups)
{
    DeviceState *st;
    if (device_state(&st) != CIO_OK) {
        return CIO_ERROR;
    }
    const uint32_t grid = workgroups ? workgroups : (uint32_t) st->cus;
    static thread_local uint32_t *sink = nullptr;
    if (!sink) {
        HIP_TRY(hipMalloc(&sink, 65536 * sizeof(uint32_t)), "read_stream: hipMalloc");
    }
    const uint64_t S = bytes / kStep;
    if (S == 0 || dev_base == nullptr) {
        return CIO_OK;
    }
    uint32_t B = 0;
    if (const char *r = cioa_diag_getenv("CIO_GPU_RS_BLOCK")) {
        B = (uint32_t) atoi(r);
    }
    if (const char *r = cioa_diag_getenv("CIO_GPU_RS_WGPOOL")) {
        const int k = atoi(r);
        if (k > 0 && k < 65536) {
            B = 0x80000000u | (uint32_t) k;
        }
    }
    unsigned long long *stamps = nullptr;
    if (const char *r = cioa_diag_getenv("CIO_GPU_RS_STAMPS")) {
        if (atoi(r) > 0) {
            if (!g_rs_stamps) {
                HIP_TRY(hipMalloc(&g_rs_stamps, 65536 * 4 * sizeof(unsigned long long)), "read_stream: hipMalloc");
            }
            stamps = g_rs_stamps;
            g_rs_waves = st->cus * (kThreads / kWave);
        }
    }
    uint32_t work = 0;
    if (const char *r = cioa_diag_getenv("CIO_GPU_RS_WORK")) {
        work = (uint32_t) std::max(0, std::min(65535, atoi(r)));
    }
    if (const char *r = cioa_diag_getenv("CIO_GPU_RS_LANE")) {
        // diagnostic: bytes per lane and step-row, 16 (coalesced rows), 32 or 64
        const int lb = atoi(r);
        work |= (lb == 64 ? 2u : lb == 32 ? 1u : 0u) << 16;
    }
#if defined(CIO_DIAG_RS_DYN)
    if (const char *r = cioa_diag_getenv("CIO_GPU_RS_DYN")) {
        unsigned pm = 0, U = 4, NC = 64;
        if (sscanf(r, "%u,%u,%u", &pm, &U, &NC) >= 1 && pm > 0 && pm <= 1000 && U >= 1 && NC >= 1 &&
            NC <= 1024) {
            static thread_local uint32_t *ctr = nullptr;
            if (!ctr) {
                HIP_TRY(hipMalloc(&ctr, 1024 * 32 * sizeof(uint32_t)), "read_stream: hipMalloc");
            }
            const uint64_t P = S * pm / 1000;
            const uint64_t npool = (P + U - 1) / U;
            const uint32_t upc = (uint32_t) ((npool + NC - 1) / NC);
            hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
            HIP_TRY(hipMemsetAsync(ctr, 0, (size_t) NC * 32 * sizeof(uint32_t), hs), "read_stream: memset");
            if (ev0) {
                HIP_TRY(hipEventRecord(ev0, hs), "hipEventRecord");
            }
            hipLaunchKernelGGL(read_stream_dyn_kernel, dim3(st->cus), dim3(kThreads), 0, hs,
                               reinterpret_cast<const uint8_t *>(dev_base), S, S - P, (uint32_t) U, ctr,
                               (uint32_t) NC, upc, (uint32_t) npool, sink);
            HIP_TRY(hipGetLastError(), "read_stream_dyn_kernel launch");
            if (ev1) {
                HIP_TRY(hipEventRecord(ev1, hs), "hipEventRecord");
            }
            return CIO_OK;
        }
    }
#endif
    if (ev0) {
        HIP_TRY(hipEventRecord(ev0, reinterpret_cast<hipStream_t>(stream)), "hipEventRecord");
    }
    hipLaunchKernelGGL(read_stream_kernel, dim3(grid), dim3(kThreads), 0,
                       reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<const uint8_t *>(dev_base), S, sink, B, stamps, work);
    HIP_TRY(hipGetLastError(), "read_stream_kernel launch");
    if (ev1) {
        HIP_TRY(hipEventRecord(ev1, reinterpret_cast<hipStream_t>(stream)), "hipEventRecord");
    }
    return CIO_OK;
}

void *cio_gpu_event_create(void)
{
    hipEvent_t ev = nullptr;
    if (hipEventCreate(&ev) != hipSuccess) {
        return nullptr;
    }
    return ev;
}

void cio_gpu_event_destroy(void *ev)
{
    if (ev) {
        (void) hipEventDestroy(reinterpret_cast<hipEvent_t>(ev));
    }
}

int cio_gpu_event_record(void *ev, void *stream)
{
    HIP_TRY(hipEventRecord(reinterpret_cast<hipEvent_t>(ev), reinterpret_cast<hipStream_t>(stream)),
            "hipEventRecord");
    return CIO_OK;
}

float cio_gpu_event_elapsed_ms(void *start, void *stop)
{
    float ms = -1.0f;
    if (hipEventSynchronize(reinterpret_cast<hipEvent_t>(stop)) != hipSuccess) {
        return -1.0f;
    }
    if (hipEventElapsedTime(&ms, reinterpret_cast<hipEvent_t>(start),
                            reinterpret_cast<hipEvent_t>(stop)) != hipSuccess) {
        return -1.0f;
    }
    return ms;
}

int cio_gpu_stream_sync(void *stream)
{
    HIP_TRY(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)), "hipStreamSynchronize");
    return CIO_OK;
}

}  // extern "C"

