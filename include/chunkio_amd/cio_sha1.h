/*
 * cio_sha1.h -- chunkio's SHA-1 wrapper as libchunkio_amd.so exports it.
 *
 * Same declarations as the reference's include/chunkio/cio_sha1.h:25-34 (and
 * the same include guard, so either header may come first):
 *
 *   struct cio_sha1 { SHA_CTX sha; }
 *   cio_sha1_init / cio_sha1_update / cio_sha1_final     src/cio_sha1.c:26-39
 *   cio_sha1_hash(data, len, out[20], state)             src/cio_sha1.c:41-57:
 *       one-shot digest; when state != NULL it receives the 96-byte SHA_CTX as
 *       it was before SHA1_Final, so hashing can go on from it
 *   cio_sha1_to_hex(in[20], out[41])                     src/cio_sha1.c:59-68
 *
 * The host SHA-1 runs on the CPU's SHA extensions where present (FIPS 180-4;
 * SHA_CTX bytes identical to OpenSSL's, see sha1/sha1.h).  Batches of chunks
 * already in HBM go to cio_sha1_batch_dev / cio_sha1_update/final_batch_dev
 * (cio_crc32_gpu.h), whose per-chunk contexts are this same SHA_CTX.
 */
#ifndef CIO_SHA1_H
#define CIO_SHA1_H

#include <sha1/sha1.h>

#ifdef __cplusplus
extern "C" {
#endif

struct cio_sha1 {
    SHA_CTX sha;
};

void cio_sha1_init(struct cio_sha1 *ctx);
void cio_sha1_update(struct cio_sha1 *ctx, const void *data, unsigned long len);
void cio_sha1_final(unsigned char hash[20], struct cio_sha1 *ctx);
void cio_sha1_hash(const void *data_in, unsigned long length,
                   unsigned char *data_out, void *state);
void cio_sha1_to_hex(unsigned char *in, char *out);

#ifdef __cplusplus
}
#endif

#endif /* CIO_SHA1_H */
