/*
 * cio_sha1.c -- host SHA-1 and chunkio's cio_sha1 wrapper (include/sha1/sha1.h,
 * include/chunkio_amd/cio_sha1.h).
 *
 * Reference: src/cio_sha1.c:26-68 wraps an un-vendored <sha1/sha1.h> whose
 * SHA_CTX / SHA1_Init / SHA1_Update / SHA1_Final API is OpenSSL's.  This file
 * is that dependency for libchunkio_amd.so, with the SHA_CTX bytes OpenSSL
 * leaves after every call (crypto/md32_common.h's update/final over
 * crypto/sha/sha_local.h's block function):
 *
 *   - Nl/Nh count BITS, low word first, carried across 2^32;
 *   - pending bytes sit raw at the front of data[], the rest of data[] is 0
 *     (a consumed partial block is zeroed, and Init zeroes everything);
 *   - Final pads (0x80, zeros, the 64-bit big-endian bit count), leaves the
 *     final chaining value and Nl/Nh in the context and zeroes data[] and num.
 *
 * Blocks run on the CPU's SHA extensions (SHA1RNDS4 / SHA1NEXTE / SHA1MSG1 /
 * SHA1MSG2) when it has them -- Zen and recent Intel cores do; 2.57 GB/s on
 * one core of the MI355X box's EPYC 9575F, OpenSSL's rate there (bench.py's
 * SHA-1 leg, library_host_path) -- else on a portable FIPS 180-4 loop.  CIOA_HOST_SHA1=portable pins
 * the portable loop (tests run both).
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <sha1/sha1.h>
#include "chunkio_amd/cio_sha1.h"
#include "crc32_host.h"

_Static_assert(sizeof(SHA_CTX) == 96, "SHA_CTX is OpenSSL's 96-byte layout");
_Static_assert(offsetof(SHA_CTX, Nl) == 20 && offsetof(SHA_CTX, data) == 28 && offsetof(SHA_CTX, num) == 92,
               "SHA_CTX field offsets are OpenSSL's");

#if defined(__x86_64__)
#include <immintrin.h>
#include <cpuid.h>
#endif

static inline uint32_t rol32(uint32_t x, int n)
{
    return (x << n) | (x >> (32 - n));
}

static inline uint32_t load_be32(const uint8_t *p)
{
    return ((uint32_t) p[0] << 24) | ((uint32_t) p[1] << 16) | ((uint32_t) p[2] << 8) | (uint32_t) p[3];
}

/* FIPS 180-4 6.1.2 over nb 64-byte blocks, a 16-word rolling schedule. */
static void blocks_portable(uint32_t h[5], const uint8_t *p, size_t nb)
{
    for (; nb > 0; nb--, p += 64) {
        uint32_t w[16];
        for (int t = 0; t < 16; t++) {
            w[t] = load_be32(p + 4 * t);
        }
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
        for (int t = 0; t < 80; t++) {
            if (t >= 16) {
                w[t & 15] = rol32(w[(t - 3) & 15] ^ w[(t - 8) & 15] ^ w[(t - 14) & 15] ^ w[t & 15], 1);
            }
            uint32_t f, k;
            if (t < 20) {
                f = (b & c) | (~b & d);
                k = 0x5A827999u;
            } else if (t < 40) {
                f = b ^ c ^ d;
                k = 0x6ED9EBA1u;
            } else if (t < 60) {
                f = (b & c) | (b & d) | (c & d);
                k = 0x8F1BBCDCu;
            } else {
                f = b ^ c ^ d;
                k = 0xCA62C1D6u;
            }
            const uint32_t tmp = rol32(a, 5) + f + e + k + w[t & 15];
            e = d;
            d = c;
            c = rol32(b, 30);
            b = a;
            a = tmp;
        }
        h[0] += a;
        h[1] += b;
        h[2] += c;
        h[3] += d;
        h[4] += e;
    }
}

#if defined(__x86_64__)
/* The same with the SHA extensions.  ABCD holds A in its top lane, E its own
 * register's top lane; each SHA1RNDS4 runs 4 rounds with the round function
 * of its immediate (0..3 = rounds 0-19, 20-39, 40-59, 60-79).  Group g (rounds
 * 4g..4g+3) uses message words W[g] = m[g % 4]; while it runs, the schedule
 * advances: W[g+1] is finished (SHA1MSG2), W[g+2] gets its XOR term and W[g+3]
 * its SHA1MSG1 term.  The E input of group g is SHA1NEXTE(ABCD of group g-1,
 * W[g]), i.e. rol(A, 30) of the state two groups back plus the words. */
#define RNDS4(abcd, e, g)                                                              \
    ((g) < 5 ? _mm_sha1rnds4_epu32(abcd, e, 0) : (g) < 10 ? _mm_sha1rnds4_epu32(abcd, e, 1) \
     : (g) < 15 ? _mm_sha1rnds4_epu32(abcd, e, 2) : _mm_sha1rnds4_epu32(abcd, e, 3))

__attribute__((target("sha,sse4.1,ssse3")))
static void blocks_shani(uint32_t h[5], const uint8_t *p, size_t nb)
{
    const __m128i bswap = _mm_set_epi64x(0x0001020304050607ll, 0x08090a0b0c0d0e0fll);
    __m128i abcd = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i *) h), 0x1B);
    __m128i e0 = _mm_set_epi32((int) h[4], 0, 0, 0);
    for (; nb > 0; nb--, p += 64) {
        const __m128i abcd_in = abcd, e_in = e0;
        __m128i m[4];
        __m128i e[2];
        for (int k = 0; k < 4; k++) {
            m[k] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *) (p + 16 * k)), bswap);
        }
        e[0] = e0;
#pragma GCC unroll 20
        for (int g = 0; g < 20; g++) {
            const __m128i w = m[g & 3];
            e[g & 1] = g == 0 ? _mm_add_epi32(e[0], w) : _mm_sha1nexte_epu32(e[g & 1], w);
            e[(g + 1) & 1] = abcd;
            if (g >= 3 && g <= 18) {
                m[(g + 1) & 3] = _mm_sha1msg2_epu32(m[(g + 1) & 3], w);
            }
            abcd = RNDS4(abcd, e[g & 1], g);
            if (g >= 1 && g <= 16) {
                m[(g - 1) & 3] = _mm_sha1msg1_epu32(m[(g - 1) & 3], w);
            }
            if (g >= 2 && g <= 17) {
                m[(g - 2) & 3] = _mm_xor_si128(m[(g - 2) & 3], w);
            }
        }
        /* after group 19 e[0] holds the ABCD group 19 started from */
        e0 = _mm_sha1nexte_epu32(e[0], e_in);
        abcd = _mm_add_epi32(abcd, abcd_in);
    }
    _mm_storeu_si128((__m128i *) h, _mm_shuffle_epi32(abcd, 0x1B));
    h[4] = (uint32_t) _mm_extract_epi32(e0, 3);
}

static int cpu_has_shani(void)
{
    unsigned a, b, c, d;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) {
        return 0;
    }
    const int sha = (b >> 29) & 1;
    if (!__get_cpuid(1, &a, &b, &c, &d)) {
        return 0;
    }
    const int sse41 = (c >> 19) & 1, ssse3 = (c >> 9) & 1;
    return sha && sse41 && ssse3;
}
#endif

typedef void (*blocks_fn)(uint32_t h[5], const uint8_t *p, size_t nb);

static blocks_fn g_blocks;

static blocks_fn pick_blocks(void)
{
    blocks_fn f = __atomic_load_n(&g_blocks, __ATOMIC_ACQUIRE);
    if (f) {
        return f;
    }
    f = blocks_portable;
#if defined(__x86_64__)
    const char *pin = cioa_diag_getenv("CIOA_HOST_SHA1");
    if (!(pin && strcmp(pin, "portable") == 0) && cpu_has_shani()) {
        f = blocks_shani;
    }
#endif
    __atomic_store_n(&g_blocks, f, __ATOMIC_RELEASE);
    return f;
}

/* Test hook (not in the public headers): pin the portable loop (1) or go back
 * to the CPU's best (0) for the rest of the process. */
void cioa_debug_host_sha1_pin(int portable)
{
    blocks_fn f = blocks_portable;
#if defined(__x86_64__)
    if (!portable && cpu_has_shani()) {
        f = blocks_shani;
    }
#endif
    (void) pick_blocks();
    __atomic_store_n(&g_blocks, f, __ATOMIC_RELEASE);
}

/* Which block function the host SHA-1 uses: "shani" or "portable". */
const char *cioa_host_sha1_path(void)
{
#if defined(__x86_64__)
    return pick_blocks() == blocks_shani ? "shani" : "portable";
#else
    return "portable";
#endif
}

static void ctx_blocks(SHA_CTX *c, const uint8_t *p, size_t nb)
{
    uint32_t h[5] = {c->h0, c->h1, c->h2, c->h3, c->h4};
    pick_blocks()(h, p, nb);
    c->h0 = h[0];
    c->h1 = h[1];
    c->h2 = h[2];
    c->h3 = h[3];
    c->h4 = h[4];
}

int cioa_SHA1_Init(SHA_CTX *c)
{
    memset(c, 0, sizeof(*c));
    c->h0 = 0x67452301u;
    c->h1 = 0xEFCDAB89u;
    c->h2 = 0x98BADCFEu;
    c->h3 = 0x10325476u;
    c->h4 = 0xC3D2E1F0u;
    return 1;
}

int cioa_SHA1_Update(SHA_CTX *c, const void *data, size_t len)
{
    const uint8_t *p = (const uint8_t *) data;
    if (len == 0) {
        return 1;
    }
    /* bit count mod 2^64, as Nl/Nh carry it */
    const uint64_t bits = (((uint64_t) c->Nh << 32) | c->Nl) + ((uint64_t) len << 3);
    c->Nl = (uint32_t) bits;
    c->Nh = (uint32_t) (bits >> 32);
    uint8_t *pend = (uint8_t *) c->data;
    size_t num = c->num & 63u;
    if (num) {
        const size_t take = 64 - num;
        if (len < take) {
            memcpy(pend + num, p, len);
            c->num = (uint32_t) (num + len);
            return 1;
        }
        memcpy(pend + num, p, take);
        ctx_blocks(c, pend, 1);
        memset(pend, 0, 64);
        c->num = 0;
        p += take;
        len -= take;
    }
    const size_t nb = len / 64;
    if (nb) {
        ctx_blocks(c, p, nb);
        p += nb * 64;
        len -= nb * 64;
    }
    if (len) {
        memcpy(pend, p, len);
        c->num = (uint32_t) len;
    }
    return 1;
}

int cioa_SHA1_Final(unsigned char *md, SHA_CTX *c)
{
    uint8_t *pend = (uint8_t *) c->data;
    size_t num = c->num & 63u;
    pend[num++] = 0x80;
    if (num > 56) {
        memset(pend + num, 0, 64 - num);
        ctx_blocks(c, pend, 1);
        num = 0;
    }
    memset(pend + num, 0, 56 - num);
    const uint32_t hi = c->Nh, lo = c->Nl;
    for (int k = 0; k < 4; k++) {
        pend[56 + k] = (uint8_t) (hi >> (24 - 8 * k));
        pend[60 + k] = (uint8_t) (lo >> (24 - 8 * k));
    }
    ctx_blocks(c, pend, 1);
    memset(pend, 0, 64);
    c->num = 0;
    const uint32_t h[5] = {c->h0, c->h1, c->h2, c->h3, c->h4};
    for (int k = 0; k < 5; k++) {
        md[4 * k + 0] = (unsigned char) (h[k] >> 24);
        md[4 * k + 1] = (unsigned char) (h[k] >> 16);
        md[4 * k + 2] = (unsigned char) (h[k] >> 8);
        md[4 * k + 3] = (unsigned char) h[k];
    }
    return 1;
}

/* ---- chunkio's wrapper (src/cio_sha1.c:26-68) ----------------------------- */

void cio_sha1_init(struct cio_sha1 *ctx)
{
    (void) cioa_SHA1_Init(&ctx->sha);
}

void cio_sha1_update(struct cio_sha1 *ctx, const void *data, unsigned long len)
{
    (void) cioa_SHA1_Update(&ctx->sha, data, (size_t) len);
}

void cio_sha1_final(unsigned char hash[20], struct cio_sha1 *ctx)
{
    (void) cioa_SHA1_Final(hash, &ctx->sha);
}

void cio_sha1_hash(const void *data_in, unsigned long length, unsigned char *data_out, void *state)
{
    SHA_CTX c;
    (void) cioa_SHA1_Init(&c);
    (void) cioa_SHA1_Update(&c, data_in, (size_t) length);
    if (state) {
        memcpy(state, &c, sizeof(c));      /* the context before Final (:52-54) */
    }
    (void) cioa_SHA1_Final(data_out, &c);
}

void cio_sha1_to_hex(unsigned char *in, char *out)
{
    static const char hex[] = "0123456789abcdef";
    for (int i = 0; i < 20; i++) {
        out[2 * i] = hex[in[i] >> 4];
        out[2 * i + 1] = hex[in[i] & 15];
    }
    out[40] = '\0';
}
