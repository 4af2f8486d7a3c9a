/*
 * Host copies into pinned staging (the host pipeline's copy workers,
 * crc32_gpu.hip CopyPool).  The staging image is written once and then read
 * by the DMA engine, never by the CPU, so its lines need not be read into the
 * cache first: 32-byte non-temporal stores skip the read-for-ownership that a
 * plain memcpy pays on every destination line, one of the three host-memory
 * streams (source read, destination read, destination write) that compete with
 * the concurrent DMA of the other slots.  CIO_GPU_NT_COPY=0 selects memcpy.
 */
#include <immintrin.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "crc32_host.h"

__attribute__((target("avx2"))) static void copy_nt_avx2(uint8_t *dst, const uint8_t *src, size_t n)
{
    size_t head = (32 - ((uintptr_t) dst & 31)) & 31;
    if (head > n) {
        head = n;
    }
    memcpy(dst, src, head);
    dst += head;
    src += head;
    n -= head;
    const size_t body = n & ~(size_t) 127;
    for (size_t i = 0; i < body; i += 128) {
        const __m256i a = _mm256_loadu_si256((const __m256i *) (src + i));
        const __m256i b = _mm256_loadu_si256((const __m256i *) (src + i + 32));
        const __m256i c = _mm256_loadu_si256((const __m256i *) (src + i + 64));
        const __m256i d = _mm256_loadu_si256((const __m256i *) (src + i + 96));
        _mm256_stream_si256((__m256i *) (dst + i), a);
        _mm256_stream_si256((__m256i *) (dst + i + 32), b);
        _mm256_stream_si256((__m256i *) (dst + i + 64), c);
        _mm256_stream_si256((__m256i *) (dst + i + 96), d);
    }
    memcpy(dst + body, src + body, n - body);
}

static int nt_enabled(void)
{
    /* Decided once; concurrent first callers compute the same value. */
    static int v = -1;
    int x = __atomic_load_n(&v, __ATOMIC_RELAXED);
    if (x < 0) {
        const char *r = cioa_diag_getenv("CIO_GPU_NT_COPY");
        __builtin_cpu_init();
        x = (r == NULL || atoi(r) != 0) && __builtin_cpu_supports("avx2");
        __atomic_store_n(&v, x, __ATOMIC_RELAXED);
    }
    return x;
}

__attribute__((visibility("hidden"))) int cioa_stage_nt(void)
{
    return nt_enabled();
}

__attribute__((visibility("hidden"))) void cioa_stage_copy(void *dst, const void *src, size_t n)
{
    if (n >= 4096 && nt_enabled()) {
        copy_nt_avx2((uint8_t *) dst, (const uint8_t *) src, n);
    } else {
        memcpy(dst, src, n);
    }
}

/* Order this thread's non-temporal stores before whatever it publishes next
 * (the copy pool's completion count, then the caller's DMA). */
__attribute__((visibility("hidden"))) void cioa_stage_fence(void)
{
    _mm_sfence();
}
