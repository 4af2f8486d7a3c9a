// sha1_gpu.hip -- batched SHA-1 content hash over independent chunks (gfx950).
//
// Reference path (fluent/chunkio): cio_sha1_init/update/final and
// cio_sha1_hash (src/cio_sha1.c:26-57) wrap an un-vendored <sha1/sha1.h>
// whose SHA_CTX / SHA1_Init / SHA1_Update / SHA1_Final API is OpenSSL's
// (include/chunkio/cio_sha1.h:52).  The algorithm is FIPS 180-4 SHA-1; the
// digest is the 20-byte big-endian output of SHA1_Final.
//
// SHA-1 cannot be split inside a message (each 64-byte block depends on the
// previous chaining value), so the unit of parallelism is one chunk per lane:
// 1024 chunks = 16 round waves.  This config is bound by the dependent round
// chain's issue rate, not by HBM; DESIGN.md reports it as such.  The message
// schedule runs on two more waves (sha1_kernel).

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <string>
#include <type_traits>
#include <vector>
#include <mutex>
#include <atomic>
#include <algorithm>
#include <stdlib.h>

#include "cio_diag.h"
#include "crc32_host.h"
#include "chunkio_amd/cio_crc32_gpu.h"

static_assert(sizeof(cio_sha1_state) == 96, "cio_sha1_state is the 96-byte C ABI layout");
static_assert(offsetof(cio_sha1_state, Nl) == 20 && offsetof(cio_sha1_state, data) == 28 &&
              offsetof(cio_sha1_state, num) == 92, "cio_sha1_state is OpenSSL's SHA_CTX layout");

namespace {

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n)
{
    return __builtin_amdgcn_alignbit(x, x, 32 - n);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x)
{
    return __builtin_bswap32(x);
}

// gfx950 three-input bit operations (one v_bitop3_b32 each).  The XOR and
// majority tables are symmetric, so operand order does not matter for them.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint32_t maj3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

// a ? b : c; table index = (a << 2) | (b << 1) | c (checked by the FIPS 180-4
// known answers in tests/test_gpu_sha1.py).
__device__ __forceinline__ uint32_t ch3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xCA);
}

struct Sha1State {
    uint32_t h0, h1, h2, h3, h4;
};

// Round function constants K_t (FIPS 180-4 §4.2.1).
__device__ __forceinline__ constexpr uint32_t sha1_k(int t)
{
    return t < 20 ? 0x5A827999u : t < 40 ? 0x6ED9EBA1u : t < 60 ? 0x8F1BBCDCu : 0xCA62C1D6u;
}

// Block j of lane's message as 16 big-endian words: content blocks, then the
// 1 or 2 padding blocks (0x80, zeros, 64-bit bit length).
__device__ __forceinline__ void message_block(const uint8_t *p, uint64_t len, uint64_t full, uint64_t j,
                                              uint32_t w[16])
{
    if (j < full) {
        const uint8_t *b = p + j * 64;
        if (((uintptr_t) b & 15u) == 0) {
            const uint4 *q = reinterpret_cast<const uint4 *>(b);
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const uint4 x = q[v];
                w[4 * v + 0] = bswap32(x.x); w[4 * v + 1] = bswap32(x.y);
                w[4 * v + 2] = bswap32(x.z); w[4 * v + 3] = bswap32(x.w);
            }
        } else {
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                w[t] = ((uint32_t) b[4 * t] << 24) | ((uint32_t) b[4 * t + 1] << 16) |
                       ((uint32_t) b[4 * t + 2] << 8) | (uint32_t) b[4 * t + 3];
            }
        }
        return;
    }
    const uint32_t rem = (uint32_t) (len - full * 64);
    const uint8_t *tail = p + full * 64;
    const uint32_t fb = (uint32_t) (j - full);
    const uint32_t nfinal = rem < 56 ? 1u : 2u;
    for (int t = 0; t < 16; ++t) {
        uint32_t word = 0;
        for (int k = 0; k < 4; ++k) {
            const uint32_t pos = fb * 64 + 4 * t + k;
            uint32_t byte = 0;
            if (pos < rem) {
                byte = tail[pos];
            } else if (pos == rem) {
                byte = 0x80u;
            }
            word = (word << 8) | byte;
        }
        w[t] = word;
    }
    if (fb == nfinal - 1) {
        const uint64_t bits = len * 8;
        w[14] = (uint32_t) (bits >> 32);
        w[15] = (uint32_t) bits;
    }
}

// Continuation (cio_sha1_update_batch_dev): block j of the virtual message
// pending(num bytes, the state's partial block) || data, as 16 big-endian
// words, byte by byte.  Only block 0 can take pending bytes (num < 64).
__device__ __forceinline__ void cont_block(const uint8_t *p, const uint8_t *pend, uint32_t num, uint64_t j,
                                           uint32_t w[16])
{
    for (int t = 0; t < 16; ++t) {
        uint32_t word = 0;
        for (int k = 0; k < 4; ++k) {
            const uint64_t pos = j * 64 + 4 * t + k;
            const uint32_t byte = pos < num ? pend[pos] : p[pos - num];
            word = (word << 8) | byte;
        }
        w[t] = word;
    }
}

// The 80 rounds of one block from its K_t + W_t rows, folded into the chaining
// value: 5 VALU per round (two rotates, v_bitop3 round function, add, add3).
// mid() runs after row kMidRow's rounds (A/B CIO_SHA1_READ_AT: where the next
// block's row reads are issued; 0 = before the block, the shipped order).
template <int kMidRow = 0, class Mid>
__device__ __forceinline__ void sha1_block_rounds(Sha1State &st, const uint4 (&rows)[20], Mid &&mid)
{
    uint32_t a = st.h0, b = st.h1, c = st.h2, d = st.h3, e = st.h4;
#pragma unroll
    for (int r = 0; r < 20; ++r) {
        if (kMidRow > 0 && r == kMidRow) {
            mid();
        }
        const uint32_t kwv[4] = {rows[r].x, rows[r].y, rows[r].z, rows[r].w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int t = 4 * r + u;
            const uint32_t f = t < 20 ? ch3(b, c, d) : (t < 40 || t >= 60) ? xor3(b, c, d) : maj3(b, c, d);
            const uint32_t tmp = rotl(a, 5) + f + e + kwv[u];
            e = d;
            d = c;
            c = rotl(b, 30);
            b = a;
            a = tmp;
        }
    }
    st.h0 += a; st.h1 += b; st.h2 += c; st.h3 += d; st.h4 += e;
}

// One workgroup = one round wave + kShaSched schedule waves for the same
// kShaChains (32) chunks, each wave alone on its SIMD.
//  - A schedule wave's 64 lanes are 64 / kShaChains block streams of those
//    chunks (lane = stream * 32 + chunk: lanes 0-31 build block j, lanes
//    32-63 block j + 1).  Each lane loads its blocks (kShaAhead in flight),
//    byte-swaps them, expands the message schedule and writes K_t + W_t for
//    the 80 rounds to LDS.
//  - The round wave runs only the dependent round chain, 5 VALU per round.
//    Its lanes 32-63 run the same chains as lanes 0-31 and their results are
//    dropped: a wave with half its lanes masked off ran the rounds and the
//    LDS reads ~15% slower (profiles/r03/sha1/ab_sha1_exec_r03j.txt,
//    ab_sha1_masked_asm_r03j.txt).
// A lone wave issues one VALU instruction per ~4 cycles
// (tools/probe/sha1_round_probe.hip: 20.35 cycles per 5-instruction round, in
// any dependency order), so a chain's floor is ~1630 cycles per block; the
// round wave alone on register-resident rows ran cfg5 in 4.65 ms.  The
// round wave reads block j + 1's 20 rows while block j's rounds run, so the
// reads' latency is hidden; what they still cost (~6% of the chain) is
// their issue and register-file writes.  Blocks are handed over kShaPer (4)
// at a time through 2 kShaPer LDS slots, one barrier per group (~0.4%).
constexpr int kShaPer = CIO_SHA1_GROUP;           // blocks handed over per barrier (4; cio_diag.h)
constexpr int kShaSched = CIO_SHA1_SCHED_WAVES;   // schedule waves (1)
constexpr int kShaChains = CIO_SHA1_CHAINS;       // chunks per workgroup, wide geometry (32)
constexpr int kShaRowsPerBlock = 20;              // 80 rounds as 20 rows of 4 (ds_read/write_b128)
constexpr int kShaAhead = 4;                      // own blocks in flight per schedule lane
constexpr int kShaThreads = 64 * (1 + kShaSched);
constexpr int kShaStreams = kShaSched * (64 / kShaChains);   // block streams over the schedule lanes
static_assert(kShaChains == 64 || kShaChains == 32 || kShaChains == 16 || kShaChains == 8, "chunks per workgroup divide a wave");
static_assert(kShaPer % kShaStreams == 0, "every schedule stream builds the same number of blocks per group");
static_assert((kShaAhead * kShaStreams) % kShaPer == 0, "a ring turn covers whole groups");
static_assert(kShaPer % 2 == 0, "the round wave's rows alternate between two register sets");

// Workgroup geometry as a template argument: C chunks per workgroup, P blocks
// handed over per barrier.  Fewer chunks per workgroup means fewer distinct
// row addresses per round-wave read (the lanes repeat the C chains) and
// measured faster while the grid still fits the chip (1024 x 400 KB:
// 8 chunks/WG with 8 blocks per barrier 4.813 ms, 16/8 4.822, 16/4 4.831,
// 32/4 4.862; profiles/r03/sha1/ab_sha1_chains_r03zu.txt), but a round wave
// then does 64/C times the work per chain, so larger batches keep 32.
// The hand-over barrier between the schedule wave and the round wave.
// Timing-only diagnostic builds (cio_diag.h CIO_SHA1_DIAG_*: wrong digests on
// purpose, tools/sha1_ab.py --diag) drop it, the round wave's row reads, or
// the schedule wave, to attribute the kernel's time to each.
__device__ __forceinline__ void sha1_barrier()
{
#if !CIO_SHA1_DIAG_NOBAR
    __syncthreads();
#endif
}

template <int C, int P>
struct ShaGeom {
    static constexpr int kChains = C;
    static constexpr int kPer = P;
    static constexpr int kSlots = 2 * P;   // one group being read, one being written
    static constexpr int kStreams = kShaSched * (64 / C);
    static_assert(C == 64 || C == 32 || C == 16 || C == 8, "chunks per workgroup divide a wave");
    static_assert(P % kStreams == 0, "every schedule stream builds the same number of blocks per group");
    static_assert((kShaAhead * kStreams) % P == 0, "a ring turn covers whole groups");
    static_assert(P % 2 == 0, "the round wave's rows alternate between two register sets");
};
using ShaGeomWide = ShaGeom<kShaChains, kShaPer>;   // the default (CIO_SHA1_CHAINS / GROUP for A/B)
using ShaGeom16 = ShaGeom<16, 8>;
using ShaGeom8 = ShaGeom<8, CIO_SHA1_GROUP8>;

#if CIO_SHA1_CLOCK_DIAG
// Diagnostic builds only: per workgroup, the round wave's shader-clock and
// 100 MHz counters at the start and the end of its block loop (read back by
// cio_sha1_diag_clock; tools/sha1_clock.py turns them into the clock the
// kernel ran at and cycles per round).
constexpr int kClkMax = 8192;
__device__ unsigned long long g_sha1_clk[kClkMax][4];
#endif

// kCont = false: one-shot digests (SHA1_Init + SHA1_Update + SHA1_Final per
// chunk).  kCont = true: SHA1_Update over a per-chunk cio_sha1_state: the
// virtual message is the state's pending bytes || the chunk's bytes; its
// whole blocks are hashed into the state's chaining value and the rest
// becomes the new pending block (no padding: sha1_final_kernel pads).
template <bool kCont, class G>
__global__ void __launch_bounds__(kShaThreads)
sha1_kernel(const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
            const uint64_t *__restrict__ lens, uint8_t *__restrict__ digests,
            cio_sha1_state *__restrict__ states, uint32_t n)
{
    constexpr int kShaChains = G::kChains;
    constexpr int kShaPer = G::kPer;
    constexpr int kShaSlots = G::kSlots;
    constexpr int kShaStreams = G::kStreams;
    __shared__ uint4 kw[kShaSlots][kShaRowsPerBlock][kShaChains];   // [slot][t / 4][chunk] = K + W for t..t+3
    const uint32_t lane = threadIdx.x & (kShaChains - 1);   // this thread's chunk in the workgroup
    const bool sched = threadIdx.x >= 64;
    const uint32_t sw = sched ? (threadIdx.x - 64) / kShaChains : 0;   // a schedule lane's block stream
    const uint32_t i = blockIdx.x * kShaChains + lane;
    const bool live = i < n;
    const uint32_t ic = live ? i : n - 1;
    const uint8_t *p = base + offs[ic];
    const uint64_t len = lens[ic];
    // pending bytes of the state (kCont); the virtual message starts num bytes before p
    const uint32_t num = kCont ? (states[ic].num & 63u) : 0u;
    const uint8_t *pend = kCont ? reinterpret_cast<const uint8_t *>(states[ic].data) : nullptr;
    const uint64_t vlen = len + num;
    const uint64_t full = vlen / 64;
    const uint64_t nblk = live ? (kCont ? full : full + ((len - full * 64) < 56 ? 1 : 2)) : 0;
    // The workgroup's largest and smallest block counts (every wave holds all
    // of its chunks): lanes past their last block idle (masked) at the end.
    uint64_t wmax = nblk, wmin = nblk;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        wmax = max(wmax, (uint64_t) __shfl_xor((unsigned long long) wmax, o));
        wmin = min(wmin, (uint64_t) __shfl_xor((unsigned long long) wmin, o));
    }
    const uint64_t ngroups = (wmax + kShaPer - 1) / kShaPer;

    if (sched && CIO_SHA1_DIAG_NOSCHED) {
        return;                 // timing-only: no message schedule, the round wave alone
    }
    if (sched) {
        // Aligned content blocks come from a kShaAhead-deep register ring
        // (this lane's block j + kShaAhead kShaStreams is requested when block
        // j is consumed): the lanes read chunks far apart, and one block of
        // prefetch did not cover the HBM latency.
        // Block j's bytes start at vbase + 64 j (vbase = p for one-shot
        // digests; p - num for a continuation, whose block 0 mixes the
        // pending bytes with the first data bytes and is gathered bytewise:
        // lo = 1 keeps every ring load inside the chunk).
        const uint8_t *vbase = p - num;
        const bool aligned = ((uintptr_t) vbase & 15u) == 0;
        const uint4 *q = reinterpret_cast<const uint4 *>(vbase);
        const uint64_t lo = num > 0 ? 1 : 0;
        constexpr uint64_t kStride = (uint64_t) kShaAhead * kShaStreams;
        uint4 nx[kShaAhead][4];
#pragma unroll
        for (int u = 0; u < kShaAhead; ++u) {
            const uint64_t ub = sw + (uint64_t) u * kShaStreams;   // this lane's u-th block
            const uint64_t b = ub < full ? ub : (full ? full - 1 : 0);
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                nx[u][v] = (aligned && full > 0 && (!kCont || b >= lo)) ? q[b * 4 + v] : make_uint4(0, 0, 0, 0);
            }
        }
        auto produce = [&](uint64_t j, uint4 (&r)[4]) {
            if (j >= nblk) {
                return;
            }
            uint32_t w[16];
            if (aligned && j < full && (!kCont || j >= lo)) {
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    w[4 * v + 0] = bswap32(r[v].x); w[4 * v + 1] = bswap32(r[v].y);
                    w[4 * v + 2] = bswap32(r[v].z); w[4 * v + 3] = bswap32(r[v].w);
                }
                const uint64_t pf = j + kStride < full ? j + kStride : full - 1;   // clamped
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    r[v] = q[pf * 4 + v];
                }
                __builtin_amdgcn_sched_barrier(0);   // keep the prefetch ahead of the schedule
            } else if (kCont) {
                if (aligned && j + kStride < full) {
                    // keep the ring slot's next block coming (block 0 took this path)
                    const uint64_t pf = j + kStride;
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        r[v] = q[pf * 4 + v];
                    }
                }
                cont_block(p, pend, num, j, w);
            } else {
                message_block(p, len, full, j, w);
            }
            uint4 *row = &kw[j % kShaSlots][0][lane];
#pragma unroll
            for (int r = 0; r < kShaRowsPerBlock; ++r) {
                uint32_t v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int t = 4 * r + u;
                    uint32_t wt;
                    if (t < 16) {
                        wt = w[t];
                    } else {
                        wt = rotl(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
                        w[t & 15] = wt;
                    }
                    v[u] = wt + sha1_k(t);
                }
                row[r * kShaChains] = make_uint4(v[0], v[1], v[2], v[3]);
            }
        };
        // Group g = blocks [g kShaPer, (g + 1) kShaPer) is in LDS before
        // barrier g: every schedule wave meets the round wave there after its
        // last block of the group, plus one final barrier that publishes
        // nothing (ngroups + 1 per wave, as the round wave's pipeline takes).
        // Unrolled so each ring slot is a fixed register set.
        for (uint64_t jb = 0; jb < ngroups * kShaPer; jb += kStride) {
#pragma unroll
            for (int u = 0; u < kShaAhead; ++u) {
                if (jb + (uint64_t) u * kShaStreams < ngroups * kShaPer) {
                    produce(jb + sw + (uint64_t) u * kShaStreams, nx[u]);
                    if ((u * kShaStreams) % kShaPer == kShaPer - kShaStreams) {
                        sha1_barrier();
                    }
                }
            }
        }
        sha1_barrier();
        return;
    }

    Sha1State st = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    if (kCont && live) {
        const cio_sha1_state &s0 = states[i];
        st = {s0.h0, s0.h1, s0.h2, s0.h3, s0.h4};
    }
    // Block-level pipeline: block j + 1's 20 rows are requested before block
    // j's rounds and land while they run.  The barrier that publishes group
    // g + 1 is taken at the start of group g's last block, once that block's
    // rows are in registers (after it the schedule waves refill group g's
    // slots).
    uint4 ra[kShaRowsPerBlock], rb[kShaRowsPerBlock];
    auto load_block = [&](uint64_t jb, uint4 (&rows)[kShaRowsPerBlock]) {
        const uint4 *row = &kw[jb % kShaSlots][0][lane];
#pragma unroll
        for (int r = 0; r < kShaRowsPerBlock; ++r) {
            rows[r] = row[r * kShaChains];
        }
    };
    // kAll: every chunk of the workgroup has block jb.  Otherwise every lane
    // still runs the rounds (the wave issues them anyway) and a lane past its
    // last block keeps its state through a select (a per-lane branch measured
    // 5% slower in round 2: the compiler then spilled rows).
    auto run_block = [&](auto kAll, uint64_t jb, const uint4 (&rows)[kShaRowsPerBlock], auto &&mid) {
        if (decltype(kAll)::value) {
            sha1_block_rounds<CIO_SHA1_READ_AT>(st, rows, mid);
            return;
        }
        Sha1State nxs = st;
        sha1_block_rounds<CIO_SHA1_READ_AT>(nxs, rows, mid);
        const bool take = jb < nblk;
        st.h0 = take ? nxs.h0 : st.h0; st.h1 = take ? nxs.h1 : st.h1; st.h2 = take ? nxs.h2 : st.h2;
        st.h3 = take ? nxs.h3 : st.h3; st.h4 = take ? nxs.h4 : st.h4;
    };
    auto run_group = [&](auto kAll, uint64_t g) {
#pragma unroll
        for (int u = 0; u < kShaPer; ++u) {
            const uint64_t jb = g * kShaPer + u;
#if !CIO_SHA1_NO_ANCHOR
            // The rounds are pure arithmetic, so the instruction selector may
            // move a block's rounds past the next block's reads (it did in the
            // select-free groups: blocks 3 and 0 then waited on reads issued
            // just before them).  The previous block's chaining value passes
            // through an empty volatile asm with a memory clobber here, so
            // those rounds end before the reads below are issued.
            asm volatile("" : "+v"(st.h0), "+v"(st.h1), "+v"(st.h2), "+v"(st.h3), "+v"(st.h4) : : "memory");
#endif
            // This block's rows (requested a block ago) have landed; waiting
            // here lets the rounds below run while 20 newer reads are out
            // (more than lgkmcnt's 4-bit count can wait past).
            __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
            if (u == kShaPer - 1) {
                sha1_barrier();
            }
            auto next_rows = [&] {
#if !CIO_SHA1_DIAG_NOREAD
                load_block(jb + 1, (u & 1) ? ra : rb);   // after the last group: read, not used
#endif
                __builtin_amdgcn_sched_barrier(0);       // the next block's reads go out here
            };
            if (CIO_SHA1_READ_AT == 0) {
                next_rows();
            }
            run_block(kAll, jb, (u & 1) ? rb : ra, next_rows);
        }
    };
    sha1_barrier();
#if CIO_SHA1_DIAG_NOREAD
    load_block(0, rb);          // both register sets read once; every block reuses them
#endif
#if CIO_SHA1_CLOCK_DIAG
    const unsigned long long clk0 = __builtin_amdgcn_s_memtime();
    const unsigned long long rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    load_block(0, ra);
    const uint64_t gall = wmin / kShaPer;   // groups every chunk has in full: no selects
    uint64_t g = 0;
    for (; g < gall; ++g) {
        run_group(std::true_type(), g);
    }
    for (; g < ngroups; ++g) {
        run_group(std::false_type(), g);
    }
#if CIO_SHA1_CLOCK_DIAG
    {
        const unsigned long long clk1 = __builtin_amdgcn_s_memtime();
        const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0 && blockIdx.x < kClkMax) {
            g_sha1_clk[blockIdx.x][0] = clk0;
            g_sha1_clk[blockIdx.x][1] = clk1;
            g_sha1_clk[blockIdx.x][2] = rt0;
            g_sha1_clk[blockIdx.x][3] = rt1;
        }
    }
#endif
    if (!live || threadIdx.x >= kShaChains) {
        return;
    }
    if (kCont) {
        // SHA1_Update's state, as OpenSSL leaves its SHA_CTX: chaining
        // value, the bit count (Nl/Nh, mod 2^64), and the tail of the virtual
        // message as the new pending bytes, the rest of data[] zero.  The
        // schedule waves read the old pending bytes only for block 0, before
        // the first barrier; with no whole block there is no barrier and this
        // wave reads them itself (tail byte k is old byte k then, read before
        // the word holding it is written).
        cio_sha1_state &s1 = states[i];
        const uint32_t rem = (uint32_t) (vlen & 63u);
        for (uint32_t wv = 0; wv < 16; ++wv) {
            uint32_t word = 0;
            for (uint32_t b = 0; b < 4; ++b) {
                const uint32_t k = 4 * wv + b;
                const uint64_t pos = full * 64 + k;
                const uint32_t byte = k < rem ? (pos < num ? pend[pos] : p[pos - num]) : 0u;
                word |= byte << (8 * b);
            }
            s1.data[wv] = word;
        }
        s1.h0 = st.h0; s1.h1 = st.h1; s1.h2 = st.h2; s1.h3 = st.h3; s1.h4 = st.h4;
        const uint64_t bits = (((uint64_t) s1.Nh << 32) | s1.Nl) + (len << 3);
        s1.Nl = (uint32_t) bits;
        s1.Nh = (uint32_t) (bits >> 32);
        s1.num = rem;
        return;
    }
    uint8_t *out = digests + (uint64_t) i * 20;
    const uint32_t h[5] = {st.h0, st.h1, st.h2, st.h3, st.h4};
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        out[4 * k + 0] = (uint8_t) (h[k] >> 24);
        out[4 * k + 1] = (uint8_t) (h[k] >> 16);
        out[4 * k + 2] = (uint8_t) (h[k] >> 8);
        out[4 * k + 3] = (uint8_t) h[k];
    }
}

// One compression of a block given as 16 big-endian words (schedule inline).
__device__ void sha1_compress_words(Sha1State &st, uint32_t w[16])
{
    uint32_t a = st.h0, b = st.h1, c = st.h2, d = st.h3, e = st.h4;
    for (int t = 0; t < 80; ++t) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = rotl(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
            w[t & 15] = wt;
        }
        const uint32_t f = t < 20 ? ch3(b, c, d) : (t < 40 || t >= 60) ? xor3(b, c, d) : maj3(b, c, d);
        const uint32_t tmp = rotl(a, 5) + f + e + wt + sha1_k(t);
        e = d;
        d = c;
        c = rotl(b, 30);
        b = a;
        a = tmp;
    }
    st.h0 += a; st.h1 += b; st.h2 += c; st.h3 += d; st.h4 += e;
}

// SHA1_Final over each state (cio_sha1_final_batch_dev): pad the pending
// bytes (0x80, zeros, the 64-bit bit count) into 1 or 2 blocks and write the
// big-endian digest.  The state is left as it was (the pre-Final context
// cio_sha1_hash exports, src/cio_sha1.c:41-57), so hashing can go on.
__global__ void sha1_final_kernel(const cio_sha1_state *__restrict__ states, uint8_t *__restrict__ digests,
                                  uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) {
        return;
    }
    const cio_sha1_state &s0 = states[i];
    Sha1State st = {s0.h0, s0.h1, s0.h2, s0.h3, s0.h4};
    const uint32_t num = s0.num & 63u;
    const uint64_t bits = ((uint64_t) s0.Nh << 32) | s0.Nl;
    const uint8_t *pend = reinterpret_cast<const uint8_t *>(s0.data);
    uint32_t w[16];
    for (int t = 0; t < 16; ++t) {
        uint32_t word = 0;
        for (int k = 0; k < 4; ++k) {
            const uint32_t pos = 4 * t + k;
            const uint32_t byte = pos < num ? pend[pos] : pos == num ? 0x80u : 0u;
            word = (word << 8) | byte;
        }
        w[t] = word;
    }
    if (num < 56) {
        w[14] = (uint32_t) (bits >> 32);
        w[15] = (uint32_t) bits;
        sha1_compress_words(st, w);
    } else {
        sha1_compress_words(st, w);
        for (int t = 0; t < 14; ++t) {
            w[t] = 0;
        }
        w[14] = (uint32_t) (bits >> 32);
        w[15] = (uint32_t) bits;
        sha1_compress_words(st, w);
    }
    uint8_t *out = digests + (uint64_t) i * 20;
    const uint32_t h[5] = {st.h0, st.h1, st.h2, st.h3, st.h4};
    for (int k = 0; k < 5; ++k) {
        out[4 * k + 0] = (uint8_t) (h[k] >> 24);
        out[4 * k + 1] = (uint8_t) (h[k] >> 16);
        out[4 * k + 2] = (uint8_t) (h[k] >> 8);
        out[4 * k + 3] = (uint8_t) h[k];
    }
}


// Chunks per workgroup for a batch of n: the fewest (8, then 16) whose grid
// still fits one workgroup per CU, else the default geometry.
// CIO_SHA1_CHUNKS_PER_WG=8|16|32 forces one (tests run every geometry).
int sha1_chunks_per_wg(size_t n)
{
    static const int forced = [] {
        const char *r = cioa_diag_getenv("CIO_SHA1_CHUNKS_PER_WG");
        const int v = r ? atoi(r) : 0;
        return (v == 8 || v == 16 || v == 32) ? v : 0;
    }();
    if (forced) {
        return forced == 32 ? kShaChains : forced;
    }
    static std::atomic<int> cus_by_dev[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
        return kShaChains;
    }
    int cus = cus_by_dev[dev].load(std::memory_order_relaxed);
    if (cus == 0) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
            return kShaChains;
        }
        cus_by_dev[dev].store(cus, std::memory_order_relaxed);
    }
    if (n <= (size_t) 8 * (size_t) cus) {
        return 8;
    }
    if (n <= (size_t) 16 * (size_t) cus) {
        return 16;
    }
    return kShaChains;
}

int sha1_launch(const void *dev_base, const uint64_t *dev_offs, const uint64_t *dev_lens, uint8_t *dev_digests,
                cio_sha1_state *dev_states, size_t n, hipStream_t s, const char *what)
{
    if (n > 0xFFFFFFFFull - 63) {
        return cioa_fail_msg(what, "too many chunks for one launch");
    }
    const uint8_t *b = reinterpret_cast<const uint8_t *>(dev_base);
    auto launch = [&](auto geom) {
        using G = decltype(geom);
        const dim3 grid((uint32_t) ((n + G::kChains - 1) / G::kChains));
        if (dev_states) {
            hipLaunchKernelGGL((sha1_kernel<true, G>), grid, dim3(kShaThreads), 0, s, b, dev_offs, dev_lens,
                               nullptr, dev_states, (uint32_t) n);
        } else {
            hipLaunchKernelGGL((sha1_kernel<false, G>), grid, dim3(kShaThreads), 0, s, b, dev_offs, dev_lens,
                               dev_digests, nullptr, (uint32_t) n);
        }
    };
    const int per_wg = sha1_chunks_per_wg(n);
    if (per_wg == 8) {
        launch(ShaGeom8());
    } else if (per_wg == 16) {
        launch(ShaGeom16());
    } else {
        launch(ShaGeomWide());
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? CIO_OK : cioa_fail_msg(what, hipGetErrorString(e));
}

}  // namespace

#if CIO_SHA1_CLOCK_DIAG
// Diagnostic builds only: copy the first nwg workgroups' clock records
// (4 x u64 each: shader clock start/end, 100 MHz start/end) to host memory.
extern "C" int cio_sha1_diag_clock(unsigned long long *out, int nwg)
{
    if (nwg < 0 || nwg > kClkMax) {
        return CIO_ERROR;
    }
    const hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sha1_clk), (size_t) nwg * 4 * sizeof(unsigned long long));
    return e == hipSuccess ? CIO_OK : cioa_fail_msg("cio_sha1_diag_clock", hipGetErrorString(e));
}
#endif

extern "C" void cio_sha1_state_init(cio_sha1_state *states, size_t n)
{
    for (size_t k = 0; k < n; k++) {
        cio_sha1_state &s0 = states[k];   // SHA1_Init: all zero, then H0..H4
        memset(&s0, 0, sizeof(s0));
        s0.h0 = 0x67452301u;
        s0.h1 = 0xEFCDAB89u;
        s0.h2 = 0x98BADCFEu;
        s0.h3 = 0x10325476u;
        s0.h4 = 0xC3D2E1F0u;
    }
}

extern "C" int cio_sha1_update_batch_dev(const void *dev_base, const uint64_t *dev_offs, const uint64_t *dev_lens,
                                         cio_sha1_state *dev_states, size_t n, void *stream)
{
    if (n == 0) {
        return CIO_OK;
    }
    if (dev_base == nullptr || dev_offs == nullptr || dev_lens == nullptr || dev_states == nullptr) {
        return cioa_fail_msg("cio_sha1_update_batch_dev", "null pointer");
    }
    if (cio_gpu_init() != CIO_OK) {
        return CIO_ERROR;
    }
    return sha1_launch(dev_base, dev_offs, dev_lens, nullptr, dev_states, n, reinterpret_cast<hipStream_t>(stream),
                       "cio_sha1_update_batch_dev: launch");
}

extern "C" int cio_sha1_final_batch_dev(const cio_sha1_state *dev_states, uint8_t *dev_digests, size_t n,
                                        void *stream)
{
    if (n == 0) {
        return CIO_OK;
    }
    if (dev_states == nullptr || dev_digests == nullptr) {
        return cioa_fail_msg("cio_sha1_final_batch_dev", "null pointer");
    }
    if (n > 0xFFFFFFFFull - 255) {
        return cioa_fail_msg("cio_sha1_final_batch_dev", "too many chunks for one launch");
    }
    if (cio_gpu_init() != CIO_OK) {
        return CIO_ERROR;
    }
    hipLaunchKernelGGL(sha1_final_kernel, dim3((uint32_t) ((n + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), dev_states, dev_digests, (uint32_t) n);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? CIO_OK : cioa_fail_msg("cio_sha1_final_batch_dev: launch", hipGetErrorString(e));
}

extern "C" int cio_sha1_batch_dev_async(const void *dev_base, const uint64_t *dev_offs, const uint64_t *dev_lens,
                                        uint8_t *dev_digests, size_t n, void *stream)
{
    if (n == 0) {
        return CIO_OK;
    }
    if (dev_base == nullptr || dev_offs == nullptr || dev_lens == nullptr || dev_digests == nullptr) {
        return cioa_fail_msg("cio_sha1_batch_dev_async", "null pointer");
    }
    if (cio_gpu_init() != CIO_OK) {
        return CIO_ERROR;
    }
    return sha1_launch(dev_base, dev_offs, dev_lens, dev_digests, nullptr, n, reinterpret_cast<hipStream_t>(stream),
                       "cio_sha1_batch_dev_async: launch");
}

extern "C" int cio_sha1_batch_dev(const void *dev_base, const uint64_t *offs, const uint64_t *lens,
                                  uint8_t *dev_digests, size_t n, void *stream)
{
    if (n == 0) {
        return CIO_OK;
    }
    if (dev_base == nullptr || offs == nullptr || lens == nullptr || dev_digests == nullptr) {
        return cioa_fail_msg("cio_sha1_batch_dev", "null pointer");
    }
    if (cio_gpu_init() != CIO_OK) {
        return CIO_ERROR;
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    uint64_t *d = nullptr;
    hipError_t e = hipMalloc(&d, 2 * n * sizeof(uint64_t));
    if (e != hipSuccess) {
        return cioa_fail_msg("cio_sha1_batch_dev: hipMalloc", hipGetErrorString(e));
    }
    e = hipMemcpyAsync(d, offs, n * sizeof(uint64_t), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) {
        e = hipMemcpyAsync(d + n, lens, n * sizeof(uint64_t), hipMemcpyHostToDevice, s);
    }
    if (e != hipSuccess) {
        (void) hipFree(d);
        return cioa_fail_msg("cio_sha1_batch_dev: copy", hipGetErrorString(e));
    }
    const int rc = sha1_launch(dev_base, d, d + n, dev_digests, nullptr, n, s, "cio_sha1_batch_dev: launch");
    e = hipStreamSynchronize(s);
    (void) hipFree(d);
    if (rc != CIO_OK) {
        return rc;
    }
    return e == hipSuccess ? CIO_OK : cioa_fail_msg("cio_sha1_batch_dev", hipGetErrorString(e));
}
