/*
 * cio_verify.c -- batched verify-on-load of chunk files (see cio_verify.h).
 *
 * Host side: header parsing and every non-CRC check of cio_file_format_check
 * (src/cio_file.c:187-294) and mmap_file (:345-493) per chunk, in the same
 * order as the reference; then ONE GPU batch (spread over the caller's
 * devices) computes the CRC of every chunk that passed
 * (cio_crc32_batch_host_multi), and the 8-byte header compare runs on the
 * host.  A batch whose regions total at most cio_crc32_cpu_max() bytes (one
 * small chunk on open/up) is CRC'd by crc_update on this thread instead
 * (crc_route.c: below the measured crossover a GPU round trip is slower).
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <time.h>
#include <unistd.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <arpa/inet.h>

#include <crc32/crc32.h>
#include "chunkio_amd/cio_crc32_gpu.h"
#include "chunkio_amd/cio_verify.h"
#include "cio_layout.h"
#include "crc32_host.h"

static unsigned long g_verify_batches;

/* Test hook (not in the public headers): how many non-empty verify batches
 * ran in this process (the chunk layer's batching is checked with it). */
unsigned long cioa_debug_verify_batches(void)
{
    return __atomic_load_n(&g_verify_batches, __ATOMIC_RELAXED);
}

int cio_file_verify_batch_multi(cio_verify_item *items, size_t n, int flags, const int *devices, int ndev)
{
    const void **bufs = NULL;
    size_t *lens = NULL, *idx = NULL, m = 0;
    uint32_t *raw = NULL;
    int rc = CIO_OK;
    const int rw = (flags & CIOA_VERIFY_WRITEBACK) != 0;

    if (n == 0) {
        return CIO_OK;
    }
    __atomic_fetch_add(&g_verify_batches, 1, __ATOMIC_RELAXED);
    if (!items) {
        return CIO_ERROR;
    }
    bufs = malloc(n * sizeof(*bufs));
    lens = malloc(n * sizeof(*lens));
    idx = malloc(n * sizeof(*idx));
    raw = malloc(n * sizeof(*raw));
    if (!bufs || !lens || !idx || !raw) {
        rc = CIO_ERROR;
        goto out;
    }
    for (size_t i = 0; i < n; i++) {
        cio_verify_item *it = &items[i];
        it->status = CIO_OK;
        it->error = 0;
        it->crc_raw = 0;
        it->meta_len = 0;
        it->content_len = 0;
        if (it->fs_size == 0) {
            /* mmap_file on an empty file (cio_file.c:388-405): only a
             * read-write open may prepare it; then cio_file_format_check
             * writes the init header and seeds crc_cur with the CRC of the
             * two meta-length bytes (:202-227). */
            if (!rw) {
                it->status = CIO_CORRUPTED;
                it->error = CIO_ERR_PERMISSION;
                continue;
            }
            if (!it->map) {
                it->status = CIO_ERROR;
                continue;
            }
            cioa_write_init_header(it->map, (flags & CIOA_VERIFY_CHECKSUM) != 0);
            it->crc_raw = (flags & CIOA_VERIFY_CHECKSUM) ? CIOA_CRC_EMPTY_RAW : 0;
            continue;
        }
        if (!it->map) {
            it->status = CIO_ERROR;
            continue;
        }
        /* mmap_file: content size first (cio_file.c:445-464) */
        const int64_t clen = cioa_st_content_len(it->map, it->fs_size, it->taint, rw);
        if (clen == -1) {
            it->status = CIO_CORRUPTED;
            it->error = CIO_ERR_BAD_FILE_SIZE;
            continue;
        }
        /* cio_file_format_check, existing file (cio_file.c:228-292) */
        if (it->map[0] != CIOA_HDR_ID_00 || it->map[1] != CIOA_HDR_ID_01) {
            it->status = CIO_CORRUPTED;
            it->error = CIO_ERR_BAD_LAYOUT;
            continue;
        }
        it->meta_len = cioa_st_meta_len(it->map);
        it->content_len = (uint64_t) clen;
        if ((uint64_t) CIOA_HDR_MIN + it->meta_len + (uint64_t) clen > it->fs_size) {
            it->status = CIO_CORRUPTED;
            it->error = CIO_ERR_BAD_FILE_SIZE;
            continue;
        }
        if (flags & CIOA_VERIFY_CHECKSUM) {
            /* region of cio_file_calculate_checksum (cio_file.c:66-94) */
            bufs[m] = it->map + CIOA_HDR_CONTENT_OFFSET;
            lens[m] = 2 + (size_t) it->meta_len + (clen > 0 ? (size_t) clen : 0);
            idx[m] = i;
            m++;
        }
    }
    if (m > 0) {
        if (cioa_crc_batch_route(bufs, lens, NULL, raw, m, devices, ndev) != CIO_OK) {
            rc = CIO_ERROR;
            goto out;
        }
        for (size_t k = 0; k < m; k++) {
            cio_verify_item *it = &items[idx[k]];
            /* crc_check = htonl(crc_finalize(crc)) in an 8-byte crc_t, 8-byte memcmp */
            crc_t check = htonl((uint32_t) crc_finalize((crc_t) raw[k]));
            if (memcmp(it->map + 2, &check, sizeof(check)) != 0) {
                it->status = CIO_CORRUPTED;
                it->error = CIO_ERR_BAD_CHECKSUM;
            } else {
                it->crc_raw = raw[k];
            }
        }
    }
out:
    free(bufs);
    free(lens);
    free(idx);
    free(raw);
    return rc;
}

int cio_file_verify_batch(cio_verify_item *items, size_t n, int flags)
{
    return cio_file_verify_batch_multi(items, n, flags, NULL, 0);
}

/* ---- verify straight from files ------------------------------------------ *
 *
 * cio_verify_paths does not map the files: the header checks pread() the 24
 * header bytes (and, for the legacy inference, the first content byte), and
 * the CRC regions go to the GPU pipeline as file ranges that its copy
 * threads pread() into pinned staging (cio_crc32_batch_fd_multi).  The bytes
 * checked are the ones a map would show; what is saved is building and
 * tearing down a page table per file (an munmap of a faulted-in 2 MB map
 * costs a TLB shootdown across every CPU the process ran on). */

struct path_job {
    const char *const *paths;
    int *fds;
    int *status, *error;
    uint32_t *crc_raw;
    uint64_t *len;             /* CRC region length (0: not checked) */
    unsigned char (*hdr)[8];   /* stored header bytes 2..9 */
    size_t lo, hi;
    int flags;
    long page;
};

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double) t.tv_sec + (double) t.tv_nsec * 1e-9;
}

static int pread_full(int fd, void *buf, size_t n, off_t off)
{
    size_t done = 0;
    while (done < n) {
        const ssize_t r = pread(fd, (char *) buf + done, n - done, off + (off_t) done);
        if (r < 0 && errno == EINTR) {
            continue;
        }
        if (r <= 0) {
            return -1;
        }
        done += (size_t) r;
    }
    return 0;
}

/* cio_file_native_open + get_size (cio_file_unix.c:396-417, 317-341), then
 * mmap_file's and cio_file_format_check's non-CRC steps in the reference's
 * order (cio_file.c:383-405, 445-464, 202-264) on the file's bytes. */
static void *check_slice(void *arg)
{
    struct path_job *j = arg;
    const int rw = (j->flags & CIOA_VERIFY_WRITEBACK) != 0;
    const int ck = (j->flags & CIOA_VERIFY_CHECKSUM) != 0;
    for (size_t i = j->lo; i < j->hi; i++) {
        struct stat sb;
        unsigned char h[CIOA_HDR_MIN];
        j->status[i] = CIO_OK;
        j->error[i] = 0;
        j->crc_raw[i] = 0;
        j->len[i] = 0;
        j->fds[i] = open(j->paths[i], rw ? O_RDWR : O_RDONLY);
        if (j->fds[i] < 0 || fstat(j->fds[i], &sb) != 0) {
            j->status[i] = CIO_ERROR;
            continue;
        }
        const size_t size = (size_t) sb.st_size;
        if (size == 0) {
            /* empty: only a read-write open prepares it (init header, crc_cur
             * = crc_update(init, "\0\0")) */
            if (!rw) {
                j->status[i] = CIO_CORRUPTED;
                j->error[i] = CIO_ERR_PERMISSION;
                continue;
            }
            cioa_write_init_header(h, ck);
            if (ck) {
                /* This call closes the file itself, so it also does what the
                 * reference's close does to a chunk prepared this way: the
                 * chunk is unsynced (cio_file.c:396), munmap_file syncs it
                 * (:317) and finalize_checksum stores htonl(crc_finalize(
                 * crc_cur)) in the 8-byte field (:116-124, :1228), i.e.
                 * 41 d9 12 ff 00 00 00 00 -- so the next verify passes. */
                const uint32_t fin = htonl((uint32_t) crc_finalize((crc_t) CIOA_CRC_EMPTY_RAW));
                memcpy(h + 2, &fin, 4);
                memset(h + 6, 0, 4);
            }
            if (posix_fallocate(j->fds[i], 0, j->page) != 0 ||
                pwrite(j->fds[i], h, CIOA_HDR_MIN, 0) != CIOA_HDR_MIN) {
                j->status[i] = CIO_ERROR;
                continue;
            }
            j->crc_raw[i] = ck ? CIOA_CRC_EMPTY_RAW : 0;
            continue;
        }
        if (size < CIOA_HDR_MIN) {
            j->status[i] = CIO_CORRUPTED;
            j->error[i] = CIO_ERR_BAD_FILE_SIZE;
            continue;
        }
        if (pread_full(j->fds[i], h, CIOA_HDR_MIN, 0) != 0) {
            j->status[i] = CIO_ERROR;
            continue;
        }
        const uint16_t meta = cioa_st_meta_len(h);
        int64_t clen = cioa_st_get_content_len_field(h);
        const size_t content_offset = CIOA_HDR_MIN + (size_t) meta;
        if (clen == 0 && size > content_offset) {          /* legacy inference (:166-176) */
            unsigned char first = 0;
            if (pread_full(j->fds[i], &first, 1, (off_t) content_offset) != 0) {
                j->status[i] = CIO_ERROR;
                continue;
            }
            if (first != 0) {
                clen = (int64_t) size - CIOA_HDR_MIN - meta;
                if (rw) {
                    unsigned char be[4];
                    cioa_st_set_content_len(h, (uint32_t) clen);
                    memcpy(be, h + CIOA_HDR_CONTENT_LEN_OFF, 4);
                    if (pwrite(j->fds[i], be, 4, CIOA_HDR_CONTENT_LEN_OFF) != 4) {
                        j->status[i] = CIO_ERROR;
                        continue;
                    }
                }
            }
        }
        if (h[0] != CIOA_HDR_ID_00 || h[1] != CIOA_HDR_ID_01) {
            j->status[i] = CIO_CORRUPTED;
            j->error[i] = CIO_ERR_BAD_LAYOUT;
            continue;
        }
        if ((uint64_t) CIOA_HDR_MIN + meta + (uint64_t) clen > size) {
            j->status[i] = CIO_CORRUPTED;
            j->error[i] = CIO_ERR_BAD_FILE_SIZE;
            continue;
        }
        if (ck) {
            j->len[i] = 2 + (uint64_t) meta + (uint64_t) clen;
            memcpy(j->hdr[i], h + 2, 8);
        }
    }
    return NULL;
}

static void *close_slice(void *arg)
{
    struct path_job *j = arg;
    for (size_t i = j->lo; i < j->hi; i++) {
        if (j->fds[i] >= 0) {
            close(j->fds[i]);
        }
        /* cio_scan_stream_files with CIO_DELETE_IRRECOVERABLE
         * (src/cio_scan.c:107-118): a chunk that failed its load as
         * CIO_CORRUPTED with a bad checksum, size or layout is deleted. */
        if ((j->flags & CIOA_VERIFY_DELETE_IRRECOVERABLE) && j->status[i] == CIO_CORRUPTED &&
            (j->error[i] == CIO_ERR_BAD_CHECKSUM || j->error[i] == CIO_ERR_BAD_FILE_SIZE ||
             j->error[i] == CIO_ERR_BAD_LAYOUT)) {
            (void) unlink(j->paths[i]);
        }
    }
    return NULL;
}

static void run_sliced(void *(*fn)(void *), struct path_job proto, size_t n)
{
    enum { MAX_T = 16 };
    struct path_job jobs[MAX_T];
    pthread_t th[MAX_T];
    int started[MAX_T] = {0};
    size_t T = n / 32 + 1;
    if (T > MAX_T) {
        T = MAX_T;
    }
    for (size_t t = 0; t < T; t++) {
        jobs[t] = proto;
        jobs[t].lo = n * t / T;
        jobs[t].hi = n * (t + 1) / T;
    }
    for (size_t t = 1; t < T; t++) {
        started[t] = pthread_create(&th[t], NULL, fn, &jobs[t]) == 0;
        if (!started[t]) {
            fn(&jobs[t]);
        }
    }
    fn(&jobs[0]);
    for (size_t t = 1; t < T; t++) {
        if (started[t]) {
            pthread_join(th[t], NULL);
        }
    }
}

int cio_verify_paths_multi(const char *const *paths, size_t n, int flags, const int *devices, int ndev,
                           int *status, int *error, uint32_t *crc_raw)
{
    int rc = CIO_OK;
    if (n == 0) {
        return CIO_OK;
    }
    if (!paths) {
        return CIO_ERROR;
    }
    int *fds = malloc(n * sizeof(int));
    int *st = malloc(n * sizeof(int));
    int *er = malloc(n * sizeof(int));
    uint32_t *cr = malloc(n * sizeof(uint32_t));
    uint64_t *len = malloc(n * sizeof(uint64_t));
    unsigned char (*hdr)[8] = malloc(n * 8);
    int *bfd = malloc(n * sizeof(int));
    uint64_t *boff = malloc(n * sizeof(uint64_t));
    size_t *blen = malloc(n * sizeof(size_t));
    size_t *bidx = malloc(n * sizeof(size_t));
    uint32_t *raw = malloc(n * sizeof(uint32_t));
    if (!fds || !st || !er || !cr || !len || !hdr || !bfd || !boff || !blen || !bidx || !raw) {
        rc = CIO_ERROR;
        goto out;
    }
    const int timing = getenv("CIO_VERIFY_TIMING") != NULL;
    const double t0 = timing ? now_s() : 0;
    struct path_job proto = {paths, fds, st, er, cr, len, hdr, 0, 0, flags, sysconf(_SC_PAGESIZE)};
    run_sliced(check_slice, proto, n);
    const double t1 = timing ? now_s() : 0;
    size_t m = 0;
    for (size_t i = 0; i < n; i++) {
        if (st[i] == CIO_OK && len[i] > 0) {
            bfd[m] = fds[i];
            boff[m] = CIOA_HDR_CONTENT_OFFSET;
            blen[m] = (size_t) len[i];
            bidx[m++] = i;
        }
    }
    if (m > 0 && cioa_crc_fd_route(bfd, boff, blen, NULL, raw, m, devices, ndev) != CIO_OK) {
        rc = CIO_ERROR;
        proto.flags &= ~CIOA_VERIFY_DELETE_IRRECOVERABLE;     /* nothing is known to be irrecoverable */
    }
    else {
        for (size_t k = 0; k < m; k++) {
            const size_t i = bidx[k];
            /* crc_check = htonl(crc_finalize(crc)) in an 8-byte crc_t, 8-byte memcmp */
            crc_t check = htonl((uint32_t) crc_finalize((crc_t) raw[k]));
            if (memcmp(hdr[i], &check, sizeof(check)) != 0) {
                st[i] = CIO_CORRUPTED;
                er[i] = CIO_ERR_BAD_CHECKSUM;
            }
            else {
                cr[i] = raw[k];
            }
        }
    }
    const double t2 = timing ? now_s() : 0;
    run_sliced(close_slice, proto, n);
    if (timing) {
        fprintf(stderr, "cio_verify_paths: %zu files, open+headers %.2f ms, CRC batch %.2f ms, close %.2f ms\n",
                n, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (now_s() - t2) * 1e3);
    }
    for (size_t i = 0; i < n; i++) {
        if (status) {
            status[i] = st[i];
        }
        if (error) {
            error[i] = er[i];
        }
        if (crc_raw) {
            crc_raw[i] = cr[i];
        }
    }
out:
    free(fds);
    free(st);
    free(er);
    free(cr);
    free(len);
    free(hdr);
    free(bfd);
    free(boff);
    free(blen);
    free(bidx);
    free(raw);
    return rc;
}

int cio_verify_paths(const char *const *paths, size_t n, int flags, int *status, int *error,
                     uint32_t *crc_raw)
{
    return cio_verify_paths_multi(paths, n, flags, NULL, 0, status, error, crc_raw);
}
