/*
 * crc32_host.c -- host-side CRC-32 math for libchunkio_amd.so.
 *
 *  - crc_update(): the host drop-in for deps/crc32/crc32.c:337-390
 *    (same contract: raw state in/out, any alignment, len 0 ok, masked to
 *    32 bits).  Carry-less-multiply folding where the CPU has it (4 x 512-bit
 *    VPCLMULQDQ accumulators from 1 KiB, 4 x 128-bit PCLMULQDQ from 64 B),
 *    slice-by-16 over tables generated at load time from the reflected
 *    polynomial otherwise and for short tails; used by chunkio's per-write
 *    path (src/cio_file.c:110) where a buffer is already in host cache, and
 *    by the chunk layer's small-batch route (crc_route.c).
 *  - GF(2) helpers: multmodp / xpow8n / shift / combine.
 *  - Generators for the device tables consumed by crc32_gpu.hip.
 */
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#include "crc32_host.h"

static uint32_t s16[16][256];
static pthread_once_t s16_once = PTHREAD_ONCE_INIT;

static void build_s16(void)
{
    for (uint32_t b = 0; b < 256; b++) {
        uint32_t c = b;
        for (int i = 0; i < 8; i++) {
            c = (c >> 1) ^ (CIOA_POLY & (0u - (c & 1u)));
        }
        s16[0][b] = c;
    }
    for (int k = 1; k < 16; k++) {
        for (uint32_t b = 0; b < 256; b++) {
            uint32_t prev = s16[k - 1][b];
            s16[k][b] = (prev >> 8) ^ s16[0][prev & 0xffu];
        }
    }
}

const uint32_t *cioa_byte_table(void)
{
    pthread_once(&s16_once, build_s16);
    return s16[0];
}

static uint32_t crc_update_table(uint32_t c, const unsigned char *p, size_t len);
static uint32_t multmodp_bits(uint32_t a, uint32_t b);

/* ---- carry-less multiply folding (x86 PCLMULQDQ / VPCLMULQDQ) -------------
 *
 * The reflected CRC as polynomial arithmetic: a 16-byte block loaded
 * little-endian into a 128-bit lane has bit k <-> x^(127-k) (bit 0 of byte 0
 * is the first message bit, the highest power).  An accumulator A (deg < 128)
 * congruent mod P to the message so far, with the state XORed into its first
 * four bytes, folds over D more bits as A x^D = A_hi x^(D+64) + A_lo x^D
 * (A_hi = low qword, A_lo = high qword).  clmul of two 64-bit reflected
 * words yields their product times x in 128-bit reflected form, so the fold
 * constants are x^(D+63) mod P (for A_hi) and x^(D-1) mod P (for A_lo), in
 * a 64-bit reflected word (coefficient of x^d at bit 63 - d).  At the end the
 * 16 bytes of A are CRC'd from state 0 by the table path: crc(0, bytes of A)
 * = A x^32 mod P, the CRC of the message.  Constants come from the same
 * GF(2) helpers as the device tables (no magic numbers). */
#if defined(__x86_64__)
#include <immintrin.h>

static uint64_t k_fold[4][2];    /* [D = 128, 512, 2048 (4 x 512-bit lanes), unused][lo, hi] */
static int have_clmul, have_vclmul;
static pthread_once_t clmul_once = PTHREAD_ONCE_INIT;

/* x^n mod P for a bit count n (reflected 32-bit: bit 31 <-> x^0). */
static uint32_t xpow_bits(uint64_t n)
{
    uint32_t r = 0x80000000u, sq = 0x40000000u;   /* x^0, x^1 */
    while (n) {
        if (n & 1u) {
            r = multmodp_bits(sq, r);
        }
        sq = multmodp_bits(sq, sq);
        n >>= 1;
    }
    return r;
}

static void build_clmul(void)
{
    const uint64_t d[3] = {128, 512, 2048};
    for (int i = 0; i < 3; i++) {
        k_fold[i][0] = (uint64_t) xpow_bits(d[i] + 63) << 32;
        k_fold[i][1] = (uint64_t) xpow_bits(d[i] - 1) << 32;
    }
    __builtin_cpu_init();
    have_clmul = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
    have_vclmul = have_clmul && __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                  __builtin_cpu_supports("vpclmulqdq");
}

__attribute__((target("pclmul,sse4.1")))
static inline __m128i fold128(__m128i x, __m128i k)
{
    return _mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11));
}

/* Bytes [0, 16 m) of p folded into one 128-bit accumulator (len >= 64). */
__attribute__((target("pclmul,sse4.1")))
static uint32_t crc_clmul(uint32_t c, const unsigned char *p, size_t len)
{
    const __m128i k128 = _mm_set_epi64x((long long) k_fold[0][1], (long long) k_fold[0][0]);
    const __m128i k512 = _mm_set_epi64x((long long) k_fold[1][1], (long long) k_fold[1][0]);
    __m128i x0 = _mm_loadu_si128((const __m128i *) p);
    __m128i x1 = _mm_loadu_si128((const __m128i *) (p + 16));
    __m128i x2 = _mm_loadu_si128((const __m128i *) (p + 32));
    __m128i x3 = _mm_loadu_si128((const __m128i *) (p + 48));
    x0 = _mm_xor_si128(x0, _mm_cvtsi32_si128((int) c));
    p += 64;
    len -= 64;
    while (len >= 64) {
        x0 = _mm_xor_si128(fold128(x0, k512), _mm_loadu_si128((const __m128i *) p));
        x1 = _mm_xor_si128(fold128(x1, k512), _mm_loadu_si128((const __m128i *) (p + 16)));
        x2 = _mm_xor_si128(fold128(x2, k512), _mm_loadu_si128((const __m128i *) (p + 32)));
        x3 = _mm_xor_si128(fold128(x3, k512), _mm_loadu_si128((const __m128i *) (p + 48)));
        p += 64;
        len -= 64;
    }
    x1 = _mm_xor_si128(fold128(x0, k128), x1);
    x2 = _mm_xor_si128(fold128(x1, k128), x2);
    x3 = _mm_xor_si128(fold128(x2, k128), x3);
    while (len >= 16) {
        x3 = _mm_xor_si128(fold128(x3, k128), _mm_loadu_si128((const __m128i *) p));
        p += 16;
        len -= 16;
    }
    unsigned char acc[16];
    _mm_storeu_si128((__m128i *) acc, x3);
    return crc_update_table(crc_update_table(0, acc, 16), p, len);
}

/* The same with four 512-bit accumulators (256 bytes per iteration), then
 * one 128-bit accumulator as above (len >= 256). */
__attribute__((target("pclmul,sse4.1,avx512f,avx512bw,vpclmulqdq")))
static uint32_t crc_vclmul(uint32_t c, const unsigned char *p, size_t len)
{
    const __m512i k2048 = _mm512_set_epi64((long long) k_fold[2][1], (long long) k_fold[2][0],
                                           (long long) k_fold[2][1], (long long) k_fold[2][0],
                                           (long long) k_fold[2][1], (long long) k_fold[2][0],
                                           (long long) k_fold[2][1], (long long) k_fold[2][0]);
    __m512i y0 = _mm512_loadu_si512((const void *) p);
    __m512i y1 = _mm512_loadu_si512((const void *) (p + 64));
    __m512i y2 = _mm512_loadu_si512((const void *) (p + 128));
    __m512i y3 = _mm512_loadu_si512((const void *) (p + 192));
    y0 = _mm512_xor_si512(y0, _mm512_zextsi128_si512(_mm_cvtsi32_si128((int) c)));
    p += 256;
    len -= 256;
    while (len >= 256) {
#define CIOA_FOLD512(y, off)                                                                         \
        y = _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(y, k2048, 0x00),                      \
                                      _mm512_clmulepi64_epi128(y, k2048, 0x11),                      \
                                      _mm512_loadu_si512((const void *) (p + (off))), 0x96)
        CIOA_FOLD512(y0, 0);
        CIOA_FOLD512(y1, 64);
        CIOA_FOLD512(y2, 128);
        CIOA_FOLD512(y3, 192);
#undef CIOA_FOLD512
        p += 256;
        len -= 256;
    }
    /* The 16 lanes of y0..y3 are 16 consecutive 16-byte blocks: fold them in
     * order into one 128-bit accumulator. */
    const __m128i k128 = _mm_set_epi64x((long long) k_fold[0][1], (long long) k_fold[0][0]);
    __m128i lanes[16];
    _mm512_storeu_si512((void *) &lanes[0], y0);
    _mm512_storeu_si512((void *) &lanes[4], y1);
    _mm512_storeu_si512((void *) &lanes[8], y2);
    _mm512_storeu_si512((void *) &lanes[12], y3);
    __m128i x = lanes[0];
    for (int i = 1; i < 16; i++) {
        x = _mm_xor_si128(fold128(x, k128), lanes[i]);
    }
    while (len >= 16) {
        x = _mm_xor_si128(fold128(x, k128), _mm_loadu_si128((const __m128i *) p));
        p += 16;
        len -= 16;
    }
    unsigned char acc[16];
    _mm_storeu_si128((__m128i *) acc, x);
    return crc_update_table(crc_update_table(0, acc, 16), p, len);
}
#endif

/* CIOA_HOST_CRC=table forces the table path (A/B and tests). */
static int host_crc_mode(void)
{
    static int mode = -1;     /* read once; concurrent first callers compute the same value */
    int m = __atomic_load_n(&mode, __ATOMIC_RELAXED);
    if (m < 0) {
        const char *r = cioa_diag_getenv("CIOA_HOST_CRC");
        m = (r && strcmp(r, "table") == 0) ? 0 : (r && strcmp(r, "clmul") == 0) ? 1 : 2;
        __atomic_store_n(&mode, m, __ATOMIC_RELAXED);
    }
    return m;
}

uint64_t cioa_crc_update_host(uint64_t crc, const void *data, size_t len)
{
    const unsigned char *p = (const unsigned char *) data;
    uint32_t c = (uint32_t) crc;

    pthread_once(&s16_once, build_s16);
    /* crc_t is 8 bytes and deps/crc32 does not mask on entry: when its first
     * byte goes through the byte loop (misaligned start, crc32.c:343-348, or
     * fewer than 8 bytes, :384-386) the shift runs on the 64-bit state, so
     * bits 32..39 land in bits 24..31; an 8-aligned word step (:366) reads
     * only the low 32 bits.  Match that, then continue on 32 bits. */
    if ((crc >> 32) && len && (((uintptr_t) p & 7u) || len < 8)) {
        c = s16[0][(crc ^ *p) & 0xffu] ^ (uint32_t) (crc >> 8);
        p++;
        len--;
    }
#if defined(__x86_64__)
    if (len >= 64) {
        pthread_once(&clmul_once, build_clmul);
        const int mode = host_crc_mode();
        if (mode == 2 && have_vclmul && len >= 1024) {
            return (uint64_t) crc_vclmul(c, p, len);
        }
        if (mode >= 1 && have_clmul) {
            return (uint64_t) crc_clmul(c, p, len);
        }
    }
#endif
    return (uint64_t) crc_update_table(c, p, len);
}

/* Slice-by-16 over the s16 tables (built by the caller). */
static uint32_t crc_update_table(uint32_t c, const unsigned char *p, size_t len)
{
    while (len && ((uintptr_t) p & 15u)) {
        c = s16[0][(c ^ *p++) & 0xffu] ^ (c >> 8);
        len--;
    }
    while (len >= 16) {
        uint32_t w0, w1, w2, w3;
        memcpy(&w0, p, 4);
        memcpy(&w1, p + 4, 4);
        memcpy(&w2, p + 8, 4);
        memcpy(&w3, p + 12, 4);
        w0 ^= c;
        c = s16[15][w0 & 0xffu] ^ s16[14][(w0 >> 8) & 0xffu] ^
            s16[13][(w0 >> 16) & 0xffu] ^ s16[12][w0 >> 24] ^
            s16[11][w1 & 0xffu] ^ s16[10][(w1 >> 8) & 0xffu] ^
            s16[9][(w1 >> 16) & 0xffu] ^ s16[8][w1 >> 24] ^
            s16[7][w2 & 0xffu] ^ s16[6][(w2 >> 8) & 0xffu] ^
            s16[5][(w2 >> 16) & 0xffu] ^ s16[4][w2 >> 24] ^
            s16[3][w3 & 0xffu] ^ s16[2][(w3 >> 8) & 0xffu] ^
            s16[1][(w3 >> 16) & 0xffu] ^ s16[0][w3 >> 24];
        p += 16;
        len -= 16;
    }
    while (len--) {
        c = s16[0][(c ^ *p++) & 0xffu] ^ (c >> 8);
    }
    return c;
}

/* a(x)*b(x) mod P(x); bit 31 carries the x^0 coefficient (reflected). */
static uint32_t multmodp_bits(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
    for (int i = 31; i >= 0; i--) {
        p ^= b & (0u - ((a >> i) & 1u));
        b = (b >> 1) ^ (CIOA_POLY & (0u - (b & 1u)));
    }
    return p;
}

#if defined(__x86_64__)
/* a * b mod P with one carry-less multiply.  In the reflected form bit k of a
 * 32-bit word is x^(31-k), so the 63-bit product P = clmul(a, b) has bit k <->
 * x^(62-k).  Its bits 31..62 (x^31..x^0) are already reduced and land at
 * bits 0..31 of P >> 31.  Its bits 0..30 (x^62..x^32) are v(x) x^32 for the
 * 32-bit message v = P << 1 (bit j <-> x^(31-j) of the message), i.e. the
 * CRC of v's four bytes from state 0: four slice-table lookups. */
static int mm_clmul;
static pthread_once_t mm_once = PTHREAD_ONCE_INIT;

static void build_mm(void)
{
    pthread_once(&s16_once, build_s16);
    __builtin_cpu_init();
    mm_clmul = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
}

__attribute__((target("pclmul,sse4.1")))
static uint32_t multmodp_clmul(uint32_t a, uint32_t b)
{
    const __m128i p = _mm_clmulepi64_si128(_mm_cvtsi32_si128((int) a), _mm_cvtsi32_si128((int) b), 0x00);
    const uint64_t q = (uint64_t) _mm_cvtsi128_si64(p);
    const uint32_t h = (uint32_t) (q >> 31);
    const uint32_t v = (uint32_t) (q << 1);
    return h ^ s16[3][v & 0xffu] ^ s16[2][(v >> 8) & 0xffu] ^ s16[1][(v >> 16) & 0xffu] ^ s16[0][v >> 24];
}
#endif

uint32_t cioa_multmodp(uint32_t a, uint32_t b)
{
#if defined(__x86_64__)
    pthread_once(&mm_once, build_mm);
    if (mm_clmul) {
        return multmodp_clmul(a, b);
    }
#endif
    return multmodp_bits(a, b);
}

/* x^(8n) mod P by square-and-multiply over the bits of n. */
uint32_t cioa_xpow8n(uint64_t n)
{
    uint32_t r = 0x80000000u;   /* x^0 */
    uint32_t sq = 0x00800000u;  /* x^8 */
    while (n) {
        if (n & 1u) {
            r = cioa_multmodp(sq, r);
        }
        sq = cioa_multmodp(sq, sq);
        n >>= 1;
    }
    return r;
}

uint32_t cio_crc32_shift(uint32_t raw_state, uint64_t nbytes)
{
    return cioa_multmodp(cioa_xpow8n(nbytes), raw_state);
}

uint32_t cio_crc32_combine(uint32_t raw_a, uint32_t raw0_b, uint64_t len_b)
{
    return cio_crc32_shift(raw_a, len_b) ^ raw0_b;
}

/*
 * Slice tables for the device word step: tab[k][b] = shift(b, k + 1), so
 * one 4-byte step is  s' = tab[3][x.b0] ^ tab[2][x.b1] ^ tab[1][x.b2] ^ tab[0][x.b3]
 * with x = s ^ word (little-endian word).
 */
void cioa_gen_slice4(uint32_t out[4][256])
{
    pthread_once(&s16_once, build_s16);
    for (int k = 0; k < 4; k++) {
        memcpy(out[k], s16[k], sizeof(out[k]));
    }
}

/* out[k][b] = shift(b << 8k, dist) = contribution of state byte k after
 * `dist` zero bytes: shift(s, dist) = XOR_k out[k][(s >> 8k) & 0xff]. */
void cioa_gen_shift_table(uint32_t out[4][256], uint64_t dist)
{
    uint32_t xp = cioa_xpow8n(dist);
    for (int k = 0; k < 4; k++) {
        for (uint32_t b = 0; b < 256; b++) {
            out[k][b] = cioa_multmodp(xp, b << (8 * k));
        }
    }
}

/* out[m] = x^(8*m) mod P for m in [0, count). */
void cioa_gen_xpow8_table(uint32_t *out, size_t count, uint64_t unit_bytes)
{
    uint32_t step = cioa_xpow8n(unit_bytes);
    uint32_t cur = 0x80000000u;
    for (size_t m = 0; m < count; m++) {
        out[m] = cur;
        cur = cioa_multmodp(step, cur);
    }
}
