/*
 * sha1/sha1.h -- the SHA-1 dependency chunkio's cio_sha1 is written against
 * (include/chunkio/cio_sha1.h:23 includes <sha1/sha1.h>; the header is not
 * vendored in fluent/chunkio), provided by libchunkio_amd.so.
 *
 * The API is the one src/cio_sha1.c:26-57 calls -- OpenSSL's:
 *
 *   SHA_CTX                                   96-byte context (cio_sha1_state.h)
 *   SHA1_Init(SHA_CTX *)                      returns 1
 *   SHA1_Update(SHA_CTX *, const void *, n)   returns 1
 *   SHA1_Final(unsigned char md[20], SHA_CTX *)  returns 1, clears the context
 *
 * With include/ on the include path ahead of the reference's, the reference's
 * own cio_sha1.h and cio_sha1.c compile unmodified and link against the
 * library (Makefile: tests/c/bin/test_sha1_ref).  The function names are
 * macros for the library's cioa_SHA1_* symbols, so a process that also loads
 * OpenSSL's libcrypto (e.g. Python's hashlib) never has two definitions of
 * SHA1_Init.  The context bytes are OpenSSL's exactly: a context can move
 * between OpenSSL, this host SHA-1 and the GPU batch calls at any split.
 * It stands in for OpenSSL's <openssl/sha.h>, so one translation unit
 * includes one of the two (both define SHA_CTX); other files of the same
 * program may use OpenSSL's freely.
 */
#ifndef CIOA_SHA1_SHA1_H
#define CIOA_SHA1_SHA1_H

#include <stddef.h>
#include <chunkio_amd/cio_sha1_state.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef cio_sha1_state SHA_CTX;

#define SHA_DIGEST_LENGTH 20
#define SHA_CBLOCK 64

#define SHA1_Init   cioa_SHA1_Init
#define SHA1_Update cioa_SHA1_Update
#define SHA1_Final  cioa_SHA1_Final

int cioa_SHA1_Init(SHA_CTX *c);
int cioa_SHA1_Update(SHA_CTX *c, const void *data, size_t len);
int cioa_SHA1_Final(unsigned char *md, SHA_CTX *c);

#ifdef __cplusplus
}
#endif

#endif /* CIOA_SHA1_SHA1_H */
