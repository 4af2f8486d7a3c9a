/*
 * crc_route.c -- where the chunk layer's host-memory CRCs run.
 *
 * A GPU pass over host memory (cio_crc32_batch_host_multi) has a fixed cost
 * per call: the plan image and the bytes go over PCIe, the kernel launches,
 * the states come back, and the caller waits on two synchronisations.  For
 * the single-chunk paths of chunkio's API -- the verify of one chunk on
 * open/up (src/cio_file.c:266-290), a full recompute after write_at or a
 * metadata move (:97-113), a deferred catch-up before a transaction -- and
 * for small batches, the library's own crc_update (crc32_host.c, the
 * drop-in for deps/crc32/crc32.c:337-390) on the calling thread finishes
 * first.  cioa_crc_batch_route() sends a batch whose total size is at most
 * cio_crc32_cpu_max() bytes there, and everything larger to the GPU.  The
 * default comes from the latency table in profiles/r03/crossover_r03b.txt
 * (tools/crossover.py on the GPU box): one chunk through the GPU host batch
 * costs 85 us at any size up to 4 KiB and 206 us at 2 MiB (its fixed cost,
 * then ~20 GB/s), while crc_update (VPCLMULQDQ folding, crc32_host.c) takes
 * 0.3 us at 16 B and 27 us at 2 MiB (~77 GB/s on cached data), so a single
 * chunk never pays for the round trip up to 8 MiB.  A batch of many chunks
 * streams through the pipelined GPU path at ~50 GB/s (PCIe-bound) against
 * one host thread's ~25 GB/s from DRAM: 85 us + B / 50 GB/s < B / 25 GB/s
 * from B ~ 4 MiB.  Results are identical either way (both compute
 * crc_update(seed, bytes)); the public cio_crc32_batch_* entry points never
 * route -- they are the GPU path.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <unistd.h>

#include <crc32/crc32.h>
#include "chunkio_amd/cio_crc32_gpu.h"
#include "crc32_host.h"

/* Bytes per call at or below which the host CRC is faster than a GPU round
 * trip (measured; see the header comment). */
#define CIOA_CPU_CRC_MAX_DEFAULT ((size_t) 4 << 20)

static size_t g_cpu_max;
static int g_cpu_max_set;

size_t cio_crc32_cpu_max(void)
{
    if (__atomic_load_n(&g_cpu_max_set, __ATOMIC_ACQUIRE)) {
        return __atomic_load_n(&g_cpu_max, __ATOMIC_RELAXED);
    }
    const char *r = getenv("CIOA_CPU_CRC_MAX");
    if (r && *r) {
        char *end = NULL;
        const unsigned long long v = strtoull(r, &end, 10);
        if (end && *end == '\0') {
            return (size_t) v;
        }
    }
    return CIOA_CPU_CRC_MAX_DEFAULT;
}

void cio_crc32_set_cpu_max(size_t bytes)
{
    __atomic_store_n(&g_cpu_max, bytes, __ATOMIC_RELAXED);
    __atomic_store_n(&g_cpu_max_set, 1, __ATOMIC_RELEASE);
}

static int route_to_cpu(const size_t *lens, size_t n)
{
    const size_t max = cio_crc32_cpu_max();
    size_t total = 0;
    for (size_t i = 0; i < n; i++) {
        total += lens[i];
        if (total > max) {
            return 0;
        }
    }
    return 1;
}

int cioa_crc_batch_route(const void *const *bufs, const size_t *lens, const uint32_t *seeds, uint32_t *out_raw,
                         size_t n, const int *devices, int ndev)
{
    if (n == 0) {
        return CIO_OK;
    }
    if (!route_to_cpu(lens, n)) {
        return cio_crc32_batch_host_multi(bufs, lens, seeds, out_raw, n, devices, ndev);
    }
    for (size_t i = 0; i < n; i++) {
        const uint32_t s = seeds ? seeds[i] : 0xffffffffu;
        out_raw[i] = (uint32_t) crc_update((crc_t) s, bufs[i], lens[i]);
    }
    return CIO_OK;
}

int cioa_crc_fd_route(const int *fds, const uint64_t *foffs, const size_t *lens, const uint32_t *seeds,
                      uint32_t *out_raw, size_t n, const int *devices, int ndev)
{
    enum { PIECE = 256 << 10 };
    if (n == 0) {
        return CIO_OK;
    }
    if (!route_to_cpu(lens, n)) {
        return cio_crc32_batch_fd_multi(fds, foffs, lens, seeds, out_raw, n, devices, ndev);
    }
    unsigned char *buf = malloc(PIECE);
    if (!buf) {
        return cioa_fail_msg("cioa_crc_fd_route", "out of memory");
    }
    int rc = CIO_OK;
    for (size_t i = 0; i < n && rc == CIO_OK; i++) {
        crc_t c = (crc_t) (seeds ? seeds[i] : 0xffffffffu);
        size_t done = 0;
        while (done < lens[i]) {
            const size_t want = lens[i] - done < PIECE ? lens[i] - done : PIECE;
            const ssize_t r = pread(fds[i], buf, want, (off_t) (foffs[i] + done));
            if (r < 0 && errno == EINTR) {
                continue;
            }
            if (r <= 0) {
                rc = cioa_fail_msg("cioa_crc_fd_route", "short read from a file source");
                break;
            }
            c = crc_update(c, buf, (size_t) r);
            done += (size_t) r;
        }
        out_raw[i] = (uint32_t) c;
    }
    free(buf);
    return rc;
}
