/*
 * cio_verify.c -- batched verify-on-load of chunk files (see cio_verify.h).
 *
 * Host side: header parsing and every non-CRC check of cio_file_format_check
 * (src/cio_file.c:187-294) and mmap_file (:345-493) per chunk, in the same
 * order as the reference; then ONE GPU batch (spread over the caller's
 * devices) computes the CRC of every chunk that passed
 * (cio_crc32_batch_host_multi), and the 8-byte header compare runs on the
 * host.  No CRC is computed on the CPU here.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <pthread.h>
#include <unistd.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <arpa/inet.h>

#include <crc32/crc32.h>
#include "chunkio_amd/cio_crc32_gpu.h"
#include "chunkio_amd/cio_verify.h"
#include "cio_layout.h"

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
        if (cio_crc32_batch_host_multi(bufs, lens, NULL, raw, m, devices, ndev) != CIO_OK) {
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

/* ---- open / map / unmap of many files on host threads ------------------ */

struct path_job {
    const char *const *paths;
    cio_verify_item *items;
    int *fds;
    size_t lo, hi;
    int flags;
    long page;
};

static int want_populate(void)
{
    static int v = -1;
    if (v < 0) {
        const char *r = getenv("CIO_VERIFY_POPULATE");
        v = r ? atoi(r) != 0 : 1;
    }
    return v;
}

/* cio_file_native_open + get_size + map (cio_file_unix.c:396-417, 317-341,
 * 74-111) for one slice of the paths.  Maps are pre-faulted (MAP_POPULATE)
 * on these threads, so the GPU pipeline's copy threads do not take a page
 * fault per 4 KiB. */
static void *open_slice(void *arg)
{
    struct path_job *j = arg;
    const int rw = (j->flags & CIOA_VERIFY_WRITEBACK) != 0;
    const int populate = want_populate() ? MAP_POPULATE : 0;
    for (size_t i = j->lo; i < j->hi; i++) {
        struct stat sb;
        cio_verify_item *it = &j->items[i];
        it->map = NULL;
        it->fs_size = 0;
        it->status = CIO_OK;
        j->fds[i] = open(j->paths[i], rw ? O_RDWR : O_RDONLY);
        if (j->fds[i] < 0 || fstat(j->fds[i], &sb) != 0) {
            it->status = CIO_ERROR;
            continue;
        }
        it->fs_size = (size_t) sb.st_size;
        if (sb.st_size > 0) {
            void *p = mmap(NULL, (size_t) sb.st_size, rw ? PROT_READ | PROT_WRITE : PROT_READ,
                           MAP_SHARED | populate, j->fds[i], 0);
            if (p == MAP_FAILED) {
                it->status = CIO_ERROR;
            }
            else {
                it->map = (unsigned char *) p;
            }
        }
        else if (rw) {
            /* mmap_file, empty file opened RW: room for the header, one page
             * (cio_file.c:398-405), then map it for the init header. */
            void *p = MAP_FAILED;
            if (posix_fallocate(j->fds[i], 0, j->page) == 0) {
                p = mmap(NULL, (size_t) j->page, PROT_READ | PROT_WRITE, MAP_SHARED, j->fds[i], 0);
            }
            if (p == MAP_FAILED) {
                it->status = CIO_ERROR;
            }
            else {
                it->map = (unsigned char *) p;
            }
        }
    }
    return NULL;
}

static void *close_slice(void *arg)
{
    struct path_job *j = arg;
    for (size_t i = j->lo; i < j->hi; i++) {
        cio_verify_item *it = &j->items[i];
        if (it->map) {
            munmap(it->map, it->fs_size ? it->fs_size : (size_t) j->page);
        }
        if (j->fds[i] >= 0) {
            close(j->fds[i]);
        }
        /* cio_scan_stream_files with CIO_DELETE_IRRECOVERABLE
         * (src/cio_scan.c:107-118): a chunk that failed its load as
         * CIO_CORRUPTED with a bad checksum, size or layout is deleted. */
        if ((j->flags & CIOA_VERIFY_DELETE_IRRECOVERABLE) && it->status == CIO_CORRUPTED &&
            (it->error == CIO_ERR_BAD_CHECKSUM || it->error == CIO_ERR_BAD_FILE_SIZE ||
             it->error == CIO_ERR_BAD_LAYOUT)) {
            (void) unlink(j->paths[i]);
        }
    }
    return NULL;
}

static void run_sliced(void *(*fn)(void *), const char *const *paths, cio_verify_item *items, int *fds,
                       size_t n, int flags)
{
    enum { MAX_T = 16 };
    struct path_job jobs[MAX_T];
    pthread_t th[MAX_T];
    int started[MAX_T] = {0};
    size_t T = n / 32 + 1;
    if (T > MAX_T) {
        T = MAX_T;
    }
    const long page = sysconf(_SC_PAGESIZE);
    for (size_t t = 0; t < T; t++) {
        jobs[t] = (struct path_job) {paths, items, fds, n * t / T, n * (t + 1) / T, flags, page};
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
    cio_verify_item *items;
    int *fds;
    uint8_t *failed;
    int rc;

    if (n == 0) {
        return CIO_OK;
    }
    if (!paths) {
        return CIO_ERROR;
    }
    items = calloc(n, sizeof(*items));
    fds = malloc(n * sizeof(*fds));
    failed = calloc(n, 1);
    if (!items || !fds || !failed) {
        free(items);
        free(fds);
        free(failed);
        return CIO_ERROR;
    }
    run_sliced(open_slice, paths, items, fds, n, flags);
    /* an item whose open/stat/map failed stays CIO_ERROR through the batch */
    for (size_t i = 0; i < n; i++) {
        failed[i] = items[i].status == CIO_ERROR;
    }
    rc = cio_file_verify_batch_multi(items, n, flags, devices, ndev);
    for (size_t i = 0; i < n; i++) {
        if (failed[i]) {
            items[i].status = CIO_ERROR;
            items[i].error = 0;
            items[i].crc_raw = 0;
        }
        if (status) {
            status[i] = items[i].status;
        }
        if (error) {
            error[i] = items[i].error;
        }
        if (crc_raw) {
            crc_raw[i] = items[i].crc_raw;
        }
    }
    if (rc != CIO_OK) {
        /* the batch did not run: nothing is known to be irrecoverable */
        flags &= ~CIOA_VERIFY_DELETE_IRRECOVERABLE;
    }
    run_sliced(close_slice, paths, items, fds, n, flags);
    free(failed);
    free(items);
    free(fds);
    return rc;
}

int cio_verify_paths(const char *const *paths, size_t n, int flags, int *status, int *error,
                     uint32_t *crc_raw)
{
    return cio_verify_paths_multi(paths, n, flags, NULL, 0, status, error, crc_raw);
}
