/*
 * cio_verify.c -- batched verify-on-load of chunk files (see cio_verify.h).
 *
 * Host side: header parsing and every non-CRC check of cio_file_format_check
 * (src/cio_file.c:187-294) and mmap_file (:345-493) per chunk, in the same
 * order as the reference; then ONE GPU batch computes the CRC of every chunk
 * that passed (cio_crc32_batch_host), and the 8-byte header compare runs on
 * the host.  No CRC is computed on the CPU here.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <unistd.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <arpa/inet.h>

#include <crc32/crc32.h>
#include "chunkio_amd/cio_crc32_gpu.h"
#include "chunkio_amd/cio_verify.h"

/* On-disk layout, include/chunkio/cio_file_st.h:151-157 */
#define HDR_ID_00             0xc1
#define HDR_ID_01             0x00
#define HDR_MIN               24
#define HDR_CONTENT_OFFSET    22
#define HDR_CONTENT_LEN_OFF   10

static uint16_t st_meta_len(const unsigned char *map)
{
    return (uint16_t) ((map[HDR_CONTENT_OFFSET] << 8) | map[HDR_CONTENT_OFFSET + 1]);
}

static void st_set_content_len(unsigned char *map, uint32_t len)
{
    map[HDR_CONTENT_LEN_OFF + 0] = (unsigned char) (len >> 24);
    map[HDR_CONTENT_LEN_OFF + 1] = (unsigned char) (len >> 16);
    map[HDR_CONTENT_LEN_OFF + 2] = (unsigned char) (len >> 8);
    map[HDR_CONTENT_LEN_OFF + 3] = (unsigned char) len;
}

/* cio_file_st_get_content_len (cio_file_st.h:219-269), including the legacy
 * inference for files written before the length field existed. */
static int64_t st_content_len(unsigned char *map, size_t size, int taint, int writeback)
{
    if (size < HDR_MIN) {
        return -1;
    }
    const size_t content_offset = HDR_CONTENT_OFFSET + 2 + st_meta_len(map);
    const unsigned char *b = map + HDR_CONTENT_LEN_OFF;
    int64_t len = ((int64_t) b[0] << 24) | ((int64_t) b[1] << 16) | ((int64_t) b[2] << 8) | b[3];
    if (!taint && len == 0 && size > content_offset) {
        if (map[content_offset] != 0x00) {
            len = (int64_t) size - HDR_MIN - st_meta_len(map);
            if (writeback) {
                st_set_content_len(map, (uint32_t) len);
            }
        }
    }
    return len;
}

int cio_file_verify_batch(cio_verify_item *items, size_t n, int flags)
{
    const void **bufs = NULL;
    size_t *lens = NULL, *idx = NULL, m = 0;
    uint32_t *raw = NULL;
    int rc = CIO_OK;

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
            /* An empty file is initialised, not verified (cio_file.c:202-227):
             * header written, crc_cur = crc_update(init, "\0\0") = 0xBE26ED00. */
            it->crc_raw = 0xBE26ED00u;
            continue;
        }
        if (!it->map) {
            it->status = CIO_CORRUPTED;
            it->error = CIO_ERR_BAD_FILE_SIZE;
            continue;
        }
        /* mmap_file: content size first (cio_file.c:445-464) */
        const int64_t clen = st_content_len(it->map, it->fs_size, it->taint,
                                            (flags & CIOA_VERIFY_WRITEBACK) != 0);
        if (clen == -1) {
            it->status = CIO_CORRUPTED;
            it->error = CIO_ERR_BAD_FILE_SIZE;
            continue;
        }
        /* cio_file_format_check, existing file (cio_file.c:228-292) */
        if (it->map[0] != HDR_ID_00 || it->map[1] != HDR_ID_01) {
            it->status = CIO_CORRUPTED;
            it->error = CIO_ERR_BAD_LAYOUT;
            continue;
        }
        it->meta_len = st_meta_len(it->map);
        it->content_len = (uint64_t) clen;
        if ((uint64_t) HDR_MIN + it->meta_len + (uint64_t) clen > it->fs_size) {
            it->status = CIO_CORRUPTED;
            it->error = CIO_ERR_BAD_FILE_SIZE;
            continue;
        }
        if (flags & CIOA_VERIFY_CHECKSUM) {
            /* region of cio_file_calculate_checksum (cio_file.c:66-94) */
            bufs[m] = it->map + HDR_CONTENT_OFFSET;
            lens[m] = 2 + (size_t) it->meta_len + (clen > 0 ? (size_t) clen : 0);
            idx[m] = i;
            m++;
        }
    }
    if (m > 0) {
        if (cio_crc32_batch_host(bufs, lens, NULL, raw, m) != CIO_OK) {
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

int cio_verify_paths(const char *const *paths, size_t n, int flags, int *status, int *error,
                     uint32_t *crc_raw)
{
    cio_verify_item *items;
    int *fds;
    int rc;
    const int wb = (flags & CIOA_VERIFY_WRITEBACK) != 0;

    if (n == 0) {
        return CIO_OK;
    }
    items = calloc(n, sizeof(*items));
    fds = malloc(n * sizeof(*fds));
    if (!items || !fds) {
        free(items);
        free(fds);
        return CIO_ERROR;
    }
    for (size_t i = 0; i < n; i++) {
        struct stat sb;
        fds[i] = open(paths[i], wb ? O_RDWR : O_RDONLY);
        if (fds[i] < 0 || fstat(fds[i], &sb) != 0) {
            items[i].status = CIO_ERROR;
            continue;
        }
        items[i].fs_size = (size_t) sb.st_size;
        if (sb.st_size > 0) {
            void *p = mmap(NULL, (size_t) sb.st_size, wb ? PROT_READ | PROT_WRITE : PROT_READ,
                           MAP_SHARED, fds[i], 0);
            items[i].map = p == MAP_FAILED ? NULL : (unsigned char *) p;
        }
    }
    rc = cio_file_verify_batch(items, n, flags);
    for (size_t i = 0; i < n; i++) {
        if (status) {
            status[i] = (fds[i] < 0) ? CIO_ERROR : items[i].status;
        }
        if (error) {
            error[i] = items[i].error;
        }
        if (crc_raw) {
            crc_raw[i] = items[i].crc_raw;
        }
        if (items[i].map) {
            munmap(items[i].map, items[i].fs_size);
        }
        if (fds[i] >= 0) {
            close(fds[i]);
        }
    }
    free(items);
    free(fds);
    return rc;
}
