/*
 * cio_sha1_state.h -- the SHA-1 context libchunkio_amd.so carries, byte for
 * byte the layout of OpenSSL's SHA_CTX (openssl/sha.h, struct SHAstate_st),
 * which is what chunkio's cio_sha1 wraps (include/chunkio/cio_sha1.h:25-27:
 * struct cio_sha1 { SHA_CTX sha; }) and what cio_sha1_hash copies out as
 * `state` before SHA1_Final (src/cio_sha1.c:52-54).
 *
 *   h0..h4   chaining value
 *   Nl, Nh   message length in BITS so far, low and high 32-bit words
 *            (pending bytes included)
 *   data     pending bytes of the partial block, raw, in message order
 *            (OpenSSL copies them in with memcpy); bytes from num on are 0
 *   num      number of pending bytes, 0..63
 *
 * 96 bytes, 4-byte aligned, plain data: a context made by OpenSSL's
 * SHA1_Init/SHA1_Update continues on the GPU batch calls
 * (cio_sha1_update/final_batch_dev) and on the library's host SHA-1
 * (include/sha1/sha1.h), and a context those produce continues in OpenSSL.
 */
#ifndef CIO_SHA1_STATE_H
#define CIO_SHA1_STATE_H

#include <stdint.h>

typedef struct cio_sha1_state {
    uint32_t h0, h1, h2, h3, h4;
    uint32_t Nl, Nh;
    uint32_t data[16];
    uint32_t num;
} cio_sha1_state;

#endif /* CIO_SHA1_STATE_H */
