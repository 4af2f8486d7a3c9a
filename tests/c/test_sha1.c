/*
 * test_sha1.c -- chunkio's cio_sha1 API from C, for tests/test_sha1_host.py.
 *
 * Built twice (Makefile):
 *   test_sha1      the library's own cio_sha1_* (include/chunkio_amd/cio_sha1.h)
 *   test_sha1_ref  the reference's include/chunkio/cio_sha1.h and
 *                  src/cio_sha1.c compiled unmodified from /root/reference
 *                  against include/sha1/sha1.h (only where it exists)
 *
 * usage: test_sha1 DATA_FILE CASE...   CASE = off:len1,len2,...
 * For each case, the message is DATA_FILE[off, off + sum(len)) fed to
 * cio_sha1_update in those pieces.  Prints, per case:
 *   ctx <96-byte context hex>          after cio_sha1_init and after each update
 *   md <digest hex> <context hex>      cio_sha1_final's digest and the context after it
 *   hash <digest hex> <state hex>      cio_sha1_hash over the whole message
 *   hex <cio_sha1_to_hex output>
 * The Python side runs the same calls on OpenSSL (libcrypto) and compares.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifdef CIOA_REF_BOUNDARY
#include <chunkio/cio_sha1.h>
#else
#include <chunkio_amd/cio_sha1.h>
#endif

static void put_hex(const void *p, size_t n)
{
    const unsigned char *b = (const unsigned char *) p;
    for (size_t i = 0; i < n; i++) {
        printf("%02x", b[i]);
    }
}

int main(int argc, char **argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s DATA_FILE off:len,len... ...\n", argv[0]);
        return 2;
    }
    FILE *f = fopen(argv[1], "rb");
    if (!f) {
        perror(argv[1]);
        return 2;
    }
    fseek(f, 0, SEEK_END);
    const long size = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char *data = malloc((size_t) size + 1);
    if (!data || fread(data, 1, (size_t) size, f) != (size_t) size) {
        fprintf(stderr, "read failed\n");
        return 2;
    }
    fclose(f);
#ifdef CIOA_REF_BOUNDARY
    printf("reference include/chunkio/cio_sha1.h + src/cio_sha1.c\n");
#endif
    printf("sizeof(struct cio_sha1) %zu\n", sizeof(struct cio_sha1));
    for (int a = 2; a < argc; a++) {
        char *spec = strdup(argv[a]);
        char *colon = strchr(spec, ':');
        if (!colon) {
            fprintf(stderr, "bad case %s\n", argv[a]);
            return 2;
        }
        *colon = '\0';
        const unsigned long off = strtoul(spec, NULL, 10);
        unsigned long pos = off;
        struct cio_sha1 ctx;
        unsigned char md[20];
        char hex[41];
        printf("case %d\n", a - 2);
        cio_sha1_init(&ctx);
        printf("ctx ");
        put_hex(&ctx, sizeof(ctx));
        printf("\n");
        for (char *tok = strtok(colon + 1, ","); tok; tok = strtok(NULL, ",")) {
            const unsigned long len = strtoul(tok, NULL, 10);
            if (pos + len > (unsigned long) size) {
                fprintf(stderr, "case %d runs past the data\n", a - 2);
                return 2;
            }
            cio_sha1_update(&ctx, data + pos, len);
            pos += len;
            printf("ctx ");
            put_hex(&ctx, sizeof(ctx));
            printf("\n");
        }
        cio_sha1_final(md, &ctx);
        printf("md ");
        put_hex(md, 20);
        printf(" ");
        put_hex(&ctx, sizeof(ctx));
        printf("\n");
        unsigned char state[96];
        memset(state, 0xAB, sizeof(state));
        cio_sha1_hash(data + off, pos - off, md, state);
        printf("hash ");
        put_hex(md, 20);
        printf(" ");
        put_hex(state, sizeof(state));
        printf("\n");
        cio_sha1_to_hex(md, hex);
        printf("hex %s\n", hex);
        free(spec);
    }
    free(data);
    return 0;
}
