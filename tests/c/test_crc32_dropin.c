/*
 * The drop-in boundary, exercised from C: a translation unit that sees only
 * what src/cio_file.c sees -- the three macros of chunkio's
 * include/chunkio/cio_crc32.h:23-27, resolving <crc32/crc32.h> to this repo's
 * include/crc32/crc32.h -- and links libchunkio_amd.so instead of the
 * reference's static cio-crc32.
 *
 * Built twice by the Makefile: with -DCIOA_REF_BOUNDARY and the reference's
 * own include/chunkio/ ahead on the include path when /root/reference is
 * present (this container: the unmodified reference header is compiled
 * against the shim), and with a restatement of the same three macros
 * otherwise (the GPU box, where the reference tree does not exist).
 *
 * The call sites replayed are cio_file.c:92 (whole region from crc_init),
 * :110 (incremental per write, raw 8-byte state memcpy'd to map+2, :111) and
 * :120-123 (finalize, htonl, 8-byte memcpy).  Expected values are the
 * reference's own: tests/fs.c:201-214 (0x41D912FF, 0x103CFA67) and the
 * header of every `tools/cio -k -p` file (0x088740E7).
 *
 * CPU only (crc_update is the scalar drop-in); run by tests/test_c_api.py.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <arpa/inet.h>

#ifdef CIOA_REF_BOUNDARY
#include <chunkio/cio_crc32.h>       /* the reference's header, unmodified */
#else
#include <crc32/crc32.h>
#define cio_crc32_init() crc_init()
#define cio_crc32_update(a, b, c) crc_update(a, b, c)
#define cio_crc32_finalize(a) crc_finalize(a)
#endif

static int failures;

#define CHECK(cond)                                                      \
    do {                                                                 \
        if (!(cond)) {                                                   \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            failures++;                                                  \
        }                                                                \
    } while (0)

static unsigned char *read_file(const char *path, size_t *size)
{
    FILE *f = fopen(path, "rb");
    if (!f) {
        return NULL;
    }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char *b = malloc((size_t) n);
    if (b && fread(b, 1, (size_t) n, f) != (size_t) n) {
        free(b);
        b = NULL;
    }
    fclose(f);
    *size = (size_t) n;
    return b;
}

int main(int argc, char **argv)
{
    size_t n400 = 0;
    unsigned char *d400;
    unsigned char map[64];
    crc_t crc, tmp;

    if (argc < 2 || !(d400 = read_file(argv[1], &n400))) {
        fprintf(stderr, "usage: %s tests/golden/400kb.txt\n", argv[0]);
        return 2;
    }
    CHECK(n400 == 409600);
    CHECK(sizeof(crc_t) == 8);                          /* LP64: 8-byte header write */
    CHECK(crc_finalize(crc_update(crc_init(), "123456789", 9)) == 0xCBF43926u);
    CHECK(crc_update(0x12345678u, "", 0) == 0x12345678u);

    /* a fresh chunk: init header, crc over the 2 meta-length bytes
     * (cio_file.c:223-226 -> :92) */
    memset(map, 0, sizeof(map));
    crc_t crc_cur = cio_crc32_init();
    crc_cur = cio_crc32_update(crc_cur, map + 22, 2);
    CHECK(crc_cur == 0xBE26ED00u);
    /* cio_chunk_sync of the empty chunk: finalize_checksum (:116-124) */
    crc = htonl(cio_crc32_finalize(crc_cur));
    memcpy(map + 2, &crc, sizeof(crc));
    CHECK(map[2] == 0x41 && map[3] == 0xD9 && map[4] == 0x12 && map[5] == 0xFF);   /* tests/fs.c:201-206 */
    CHECK(map[6] == 0 && map[7] == 0 && map[8] == 0 && map[9] == 0);

    /* one 400 KB write (update_checksum :110-112), then sync: tests/fs.c:209-214 */
    crc_cur = cio_crc32_update(crc_cur, d400, n400);
    memcpy(map + 2, &crc_cur, sizeof(crc_cur));          /* raw 8-byte state, host order */
    CHECK(map[6] == 0 && map[7] == 0 && map[8] == 0 && map[9] == 0);
    CHECK(cio_crc32_finalize(crc_cur) == 0x103CFA67u);

    /* four more writes: the `cio -k -p` perf file */
    for (int i = 0; i < 4; i++) {
        crc_cur = cio_crc32_update(crc_cur, d400, n400);
    }
    crc = htonl(cio_crc32_finalize(crc_cur));
    memcpy(map + 2, &crc, sizeof(crc));
    CHECK(map[2] == 0x08 && map[3] == 0x87 && map[4] == 0x40 && map[5] == 0xE7);

    /* whole-region recompute == incremental (cio_file.c:92 vs :110), at
     * every misalignment of the region start (map + 22 is 6 mod 16) */
    unsigned char *buf = malloc(n400 + 64);
    for (int mis = 0; mis < 16; mis++) {
        memcpy(buf + mis, d400, n400);
        tmp = cio_crc32_update(cio_crc32_init(), buf + mis, n400);
        CHECK(cio_crc32_finalize(tmp) == 0x777A8F30u);
    }
    free(buf);

    /* crc_t states with bits 32..63 set (crc32.c does not mask on entry):
     * the first byte-wise step -- misaligned start (:343-348) or fewer than
     * 8 bytes (:384-386) -- shifts the 64-bit state, an 8-aligned word step
     * (:366) reads its low 32 bits.  Checked against a bitwise restatement. */
    {
        static const uint64_t wide[] = {0x1FFFFFFFFull, 0xFFFFFFFF12345678ull, 0xABCD00000000ABCDull,
                                        0xFFFFFFFFFFFFFFFFull, 0x0000000100000000ull};
        static const size_t lens[] = {0, 1, 2, 3, 7, 8, 9, 15, 16, 17, 63, 64, 65, 1023, 1024, 4093, 409600};
        unsigned char *al = aligned_alloc(64, n400 + 64);
        memcpy(al + 8, d400, n400);
        for (size_t s = 0; s < sizeof(wide) / sizeof(wide[0]); s++) {
            for (int mis = 0; mis < 8; mis++) {
                for (size_t l = 0; l < sizeof(lens) / sizeof(lens[0]); l++) {
                    const unsigned char *p = al + 8 + mis;
                    size_t len = lens[l];
                    uint64_t want = wide[s];
                    size_t i = 0;
                    if (len && (mis || len < 8)) {
                        want ^= p[0];
                        for (int b = 0; b < 8; b++) {
                            want = (want >> 1) ^ (0xEDB88320u & (0u - (unsigned) (want & 1u)));
                        }
                        i = 1;
                    }
                    want &= 0xffffffffu;
                    for (; i < len; i++) {
                        want ^= p[i];
                        for (int b = 0; b < 8; b++) {
                            want = (want >> 1) ^ (0xEDB88320u & (0u - (unsigned) (want & 1u)));
                        }
                    }
                    crc_t got = cio_crc32_update((crc_t) wide[s], p, len);
                    if ((uint64_t) got != want) {
                        fprintf(stderr, "wide seed %#llx mis %d len %zu: %#llx != %#llx\n",
                                (unsigned long long) wide[s], mis, len, (unsigned long long) got,
                                (unsigned long long) want);
                        failures++;
                    }
                }
            }
        }
        free(al);
    }
    free(d400);
    if (failures) {
        fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    printf("dropin ok%s\n",
#ifdef CIOA_REF_BOUNDARY
           " (reference include/chunkio/cio_crc32.h)"
#else
           ""
#endif
    );
    return 0;
}
