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
#include <stdint.h>
#include <string>
#include <vector>

#include "crc32_host.h"
#include "chunkio_amd/cio_crc32_gpu.h"

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

// The 80 rounds of one block from its K_t + W_t rows, folded into the chaining
// value: 5 VALU per round (two rotates, v_bitop3 round function, add, add3).
__device__ __forceinline__ void sha1_block_rounds(Sha1State &st, const uint4 (&rows)[20])
{
    uint32_t a = st.h0, b = st.h1, c = st.h2, d = st.h3, e = st.h4;
#pragma unroll
    for (int r = 0; r < 20; ++r) {
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

// One workgroup = one round wave + kShaSched schedule waves for the same 64
// chunks (one chunk per lane), each wave alone on its SIMD.
//  - Schedule wave s loads blocks j = s, s + kShaSched, ... (kShaAhead of its
//    own blocks in flight), byte-swaps them, expands the message schedule and
//    writes K_t + W_t for the 80 rounds to LDS.
//  - The round wave runs only the dependent round chain, 5 VALU per round.
// A lone wave issues one VALU instruction per ~4 cycles
// (tools/probe/sha1_round_probe.hip: 20.35 cycles per 5-instruction round, in
// any dependency order), so a chain's floor is ~1630 cycles per block.  One
// schedule wave needed more than that per block (~250 instructions plus its
// LDS writes: a build whose round wave did no rounds took 4.5 ms per cfg5
// batch), so it, not the chain, set the pace; two schedule waves halve it.
// Blocks are handed over kShaPer (4) at a time through 2 kShaPer LDS slots
// (160 KiB), one barrier per group (a barrier per block cost ~3 cycles per
// round).
#ifdef CIO_SHA1_GROUP
constexpr int kShaPer = CIO_SHA1_GROUP;           // blocks handed over per barrier
#else
constexpr int kShaPer = 4;
#endif
#ifdef CIO_SHA1_SCHED_WAVES
constexpr int kShaSched = CIO_SHA1_SCHED_WAVES;   // schedule waves
#else
constexpr int kShaSched = 2;
#endif
constexpr int kShaRowsPerBlock = 20;              // 80 rounds as 20 rows of 4 (ds_read/write_b128)
constexpr int kShaAhead = 4;                      // own blocks in flight per schedule wave
constexpr int kShaSlots = 2 * kShaPer;            // one group being read, one being written
constexpr int kShaThreads = 64 * (1 + kShaSched);
static_assert(kShaPer % kShaSched == 0, "every schedule wave builds the same number of blocks per group");
static_assert((kShaAhead * kShaSched) % kShaPer == 0, "a ring turn covers whole groups");

__global__ void __launch_bounds__(kShaThreads)
sha1_kernel(const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
            const uint64_t *__restrict__ lens, uint8_t *__restrict__ digests, uint32_t n)
{
    __shared__ uint4 kw[kShaSlots][kShaRowsPerBlock][64];   // [slot][t / 4][lane] = K + W for t..t+3
    const uint32_t lane = threadIdx.x & 63u;
    const bool sched = threadIdx.x >= 64;
    const uint32_t sw = sched ? (threadIdx.x >> 6) - 1 : 0;   // this schedule wave's block residue
    const uint32_t i = blockIdx.x * 64 + lane;
    const bool live = i < n;
    const uint32_t ic = live ? i : n - 1;
    const uint8_t *p = base + offs[ic];
    const uint64_t len = lens[ic];
    const uint64_t full = len / 64;
    const uint64_t nblk = live ? full + ((len - full * 64) < 56 ? 1 : 2) : 0;
    // The wave's block count: lanes with fewer blocks idle (masked) at the end.
    uint64_t wmax = nblk;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        wmax = max(wmax, (uint64_t) __shfl_xor((unsigned long long) wmax, o));
    }
    const uint64_t ngroups = (wmax + kShaPer - 1) / kShaPer;

    if (sched) {
        // Aligned content blocks come from a kShaAhead-deep register ring
        // (this wave's block j + kShaAhead kShaSched is requested when block j
        // is consumed): the 64 lanes read 64 chunks far apart, and one block
        // of prefetch did not cover the HBM latency.
        const bool aligned = ((uintptr_t) p & 15u) == 0;
        const uint4 *q = reinterpret_cast<const uint4 *>(p);
        constexpr uint64_t kStride = (uint64_t) kShaAhead * kShaSched;
        uint4 nx[kShaAhead][4];
#pragma unroll
        for (int u = 0; u < kShaAhead; ++u) {
            const uint64_t ub = sw + (uint64_t) u * kShaSched;   // this wave's u-th block
            const uint64_t b = ub < full ? ub : (full ? full - 1 : 0);
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                nx[u][v] = (aligned && full > 0) ? q[b * 4 + v] : make_uint4(0, 0, 0, 0);
            }
        }
        auto produce = [&](uint64_t j, uint4 (&r)[4]) {
            if (j >= nblk) {
                return;
            }
            uint32_t w[16];
            if (aligned && j < full) {
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
                row[r * 64] = make_uint4(v[0], v[1], v[2], v[3]);
            }
        };
        // Group g = blocks [g kShaPer, (g + 1) kShaPer) is in LDS before
        // barrier g: every schedule wave meets the round wave there after its
        // last block of the group (ngroups barriers per wave).  Unrolled so
        // each ring slot is a fixed register set.
        for (uint64_t jb = 0; jb < ngroups * kShaPer; jb += kStride) {
#pragma unroll
            for (int u = 0; u < kShaAhead; ++u) {
                if (jb + (uint64_t) u * kShaSched < ngroups * kShaPer) {
                    produce(jb + sw + (uint64_t) u * kShaSched, nx[u]);
                    if ((u * kShaSched) % kShaPer == kShaPer - kShaSched) {
                        __syncthreads();
                    }
                }
            }
        }
        return;
    }

    Sha1State st = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    auto load_group = [&](uint64_t g, uint4 (&rows)[kShaPer][kShaRowsPerBlock]) {
#pragma unroll
        for (int u = 0; u < kShaPer; ++u) {
            const uint4 *row = &kw[(g * kShaPer + u) % kShaSlots][0][lane];
#pragma unroll
            for (int r = 0; r < kShaRowsPerBlock; ++r) {
                rows[u][r] = row[r * 64];
            }
        }
    };
    auto run_group = [&](uint64_t g, const uint4 (&rows)[kShaPer][kShaRowsPerBlock]) {
#pragma unroll
        for (int u = 0; u < kShaPer; ++u) {
            // Every lane runs the rounds (the wave issues them anyway) and a
            // lane past its last block keeps its state: no branch for the
            // compiler to sink the row reads into, so they stay in order.
            // (A per-lane branch instead measured 5% slower: the compiler
            // then spilled rows to AGPRs, sha1_ab_branch.txt.)
            Sha1State nxs = st;
            sha1_block_rounds(nxs, rows[u]);
            const bool take = g * kShaPer + u < nblk;
            st.h0 = take ? nxs.h0 : st.h0; st.h1 = take ? nxs.h1 : st.h1; st.h2 = take ? nxs.h2 : st.h2;
            st.h3 = take ? nxs.h3 : st.h3; st.h4 = take ? nxs.h4 : st.h4;
        }
    };
    for (uint64_t g = 0; g < ngroups; ++g) {
        __syncthreads();
        // All 20 rows of every block of the group are requested up front, so
        // the LDS latency after the barrier is paid once per group.
        uint4 rows[kShaPer][kShaRowsPerBlock];
        load_group(g, rows);
        // Every row lands before the rounds start: LDS data arriving while the
        // round chain issues slows the chain more than the wait costs
        // (profiles/r02/sha1/sha1_ab_wait.txt, sha1_ab_ahead.txt).
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
        run_group(g, rows);
    }
    if (!live) {
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

}  // namespace

namespace {

int sha1_launch(const void *dev_base, const uint64_t *dev_offs, const uint64_t *dev_lens, uint8_t *dev_digests,
                size_t n, hipStream_t s)
{
    if (n > 0xFFFFFFFFull - 63) {
        return cioa_fail_msg("cio_sha1_batch_dev", "too many chunks for one launch");
    }
    hipLaunchKernelGGL(sha1_kernel, dim3((uint32_t) ((n + 63) / 64)), dim3(kShaThreads), 0, s,
                       reinterpret_cast<const uint8_t *>(dev_base), dev_offs, dev_lens, dev_digests, (uint32_t) n);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? CIO_OK : cioa_fail_msg("cio_sha1_batch_dev: launch", hipGetErrorString(e));
}

}  // namespace

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
    return sha1_launch(dev_base, dev_offs, dev_lens, dev_digests, n, reinterpret_cast<hipStream_t>(stream));
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
    const int rc = sha1_launch(dev_base, d, d + n, dev_digests, n, s);
    e = hipStreamSynchronize(s);
    (void) hipFree(d);
    if (rc != CIO_OK) {
        return rc;
    }
    return e == hipSuccess ? CIO_OK : cioa_fail_msg("cio_sha1_batch_dev", hipGetErrorString(e));
}
