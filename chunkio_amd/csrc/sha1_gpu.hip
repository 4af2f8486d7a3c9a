// sha1_gpu.hip -- batched SHA-1 content hash over independent chunks (gfx950).
//
// Reference path (fluent/chunkio): cio_sha1_init/update/final and
// cio_sha1_hash (src/cio_sha1.c:91-122) wrap an un-vendored <sha1/sha1.h>
// whose SHA_CTX / SHA1_Init / SHA1_Update / SHA1_Final API is OpenSSL's
// (include/chunkio/cio_sha1.h:52).  The algorithm is FIPS 180-4 SHA-1; the
// digest is the 20-byte big-endian output of SHA1_Final.
//
// SHA-1 cannot be split inside a message (each 64-byte block depends on the
// previous chaining value), so the unit of parallelism is one chunk per lane:
// 1024 chunks = 16 waves.  This config is latency-bound on the dependent
// round chain, not on HBM; DESIGN.md reports it as such.

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

__device__ __forceinline__ void sha1_block(Sha1State &st, uint32_t w[16])
{
    uint32_t a = st.h0, b = st.h1, c = st.h2, d = st.h3, e = st.h4;
#pragma unroll
    for (int t = 0; t < 80; ++t) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = rotl(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
            w[t & 15] = wt;
        }
        uint32_t f, k;
        if (t < 20) {
            f = ch3(b, c, d);                 // Ch
            k = 0x5A827999u;
        } else if (t < 40) {
            f = xor3(b, c, d);                // Parity
            k = 0x6ED9EBA1u;
        } else if (t < 60) {
            f = maj3(b, c, d);                // Maj
            k = 0x8F1BBCDCu;
        } else {
            f = xor3(b, c, d);
            k = 0xCA62C1D6u;
        }
        const uint32_t tmp = rotl(a, 5) + f + e + k + wt;
        e = d;
        d = c;
        c = rotl(b, 30);
        b = a;
        a = tmp;
    }
    st.h0 += a; st.h1 += b; st.h2 += c; st.h3 += d; st.h4 += e;
}

__global__ void __launch_bounds__(64)
sha1_kernel(const uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
            const uint64_t *__restrict__ lens, uint8_t *__restrict__ digests, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) {
        return;
    }
    const uint8_t *p = base + offs[i];
    const uint64_t len = lens[i];
    Sha1State st = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    uint32_t w[16];
    const uint64_t full = len / 64;
    if (((uintptr_t) p & 15u) == 0) {
        // Aligned: block b+1 is loaded while block b is hashed (one wave per
        // SIMD here, so nothing else would hide the HBM latency).
        const uint4 *q = reinterpret_cast<const uint4 *>(p);
        uint4 nx[4];
        if (full > 0) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                nx[v] = q[v];
            }
        }
        for (uint64_t blk = 0; blk < full; ++blk) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                w[4 * v + 0] = bswap32(nx[v].x); w[4 * v + 1] = bswap32(nx[v].y);
                w[4 * v + 2] = bswap32(nx[v].z); w[4 * v + 3] = bswap32(nx[v].w);
            }
            const uint64_t pf = blk + 1 < full ? blk + 1 : blk;   // clamped: always in bounds
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                nx[v] = q[pf * 4 + v];
            }
            __builtin_amdgcn_sched_barrier(0);   // keep the prefetch ahead of the rounds
            sha1_block(st, w);
        }
    } else {
        for (uint64_t blk = 0; blk < full; ++blk) {
            const uint8_t *b = p + blk * 64;
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                w[t] = ((uint32_t) b[4 * t] << 24) | ((uint32_t) b[4 * t + 1] << 16) |
                       ((uint32_t) b[4 * t + 2] << 8) | (uint32_t) b[4 * t + 3];
            }
            sha1_block(st, w);
        }
    }
    // Final block(s): remaining bytes, 0x80, zero pad, 64-bit big-endian bit length.
    const uint32_t rem = (uint32_t) (len - full * 64);
    const uint8_t *tail = p + full * 64;
    const uint64_t bits = len * 8;
    const int nfinal = rem < 56 ? 1 : 2;
    for (int fb = 0; fb < nfinal; ++fb) {
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            uint32_t word = 0;
            for (int k = 0; k < 4; ++k) {
                const uint32_t pos = (uint32_t) (fb * 64 + 4 * t + k);
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
            w[14] = (uint32_t) (bits >> 32);
            w[15] = (uint32_t) bits;
        }
        sha1_block(st, w);
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

extern "C" int cio_sha1_batch_dev(const void *dev_base, const uint64_t *offs, const uint64_t *lens,
                                  uint8_t *dev_digests, size_t n, void *stream)
{
    if (n == 0) {
        return CIO_OK;
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
    if (e == hipSuccess) {
        hipLaunchKernelGGL(sha1_kernel, dim3((uint32_t) ((n + 63) / 64)), dim3(64), 0, s,
                           reinterpret_cast<const uint8_t *>(dev_base), d, d + n, dev_digests,
                           (uint32_t) n);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        e = hipStreamSynchronize(s);
    }
    (void) hipFree(d);
    return e == hipSuccess ? CIO_OK : cioa_fail_msg("cio_sha1_batch_dev", hipGetErrorString(e));
}
