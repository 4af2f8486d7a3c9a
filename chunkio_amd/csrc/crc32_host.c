/*
 * crc32_host.c -- host-side CRC-32 math for libchunkio_amd.so.
 *
 *  - crc_update(): the scalar drop-in for deps/crc32/crc32.c:337-390
 *    (same contract: raw state in/out, any alignment, len 0 ok, masked to
 *    32 bits).  Slice-by-16 over tables generated at load time from the
 *    reflected polynomial; used by chunkio's per-write path
 *    (src/cio_file.c:110) where a buffer is already in host cache.
 *  - GF(2) helpers: multmodp / xpow8n / shift / combine.
 *  - Generators for the device tables consumed by crc32_gpu.hip.
 */
#include <stdint.h>
#include <stddef.h>
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

uint64_t cioa_crc_update_host(uint64_t crc, const void *data, size_t len)
{
    const unsigned char *p = (const unsigned char *) data;
    uint32_t c = (uint32_t) crc;

    pthread_once(&s16_once, build_s16);

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
    return (uint64_t) c;
}

/* a(x)*b(x) mod P(x); bit 31 carries the x^0 coefficient (reflected). */
uint32_t cioa_multmodp(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
    for (int i = 31; i >= 0; i--) {
        p ^= b & (0u - ((a >> i) & 1u));
        b = (b >> 1) ^ (CIOA_POLY & (0u - (b & 1u)));
    }
    return p;
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
