/*
 * cio_sync.c -- batched sync of chunk files with deferred CRC (see cio_sync.h).
 *
 * Host side: header checks and range setup per chunk, ONE GPU batch
 * (cio_crc32_batch_host, seeded with each chunk's crc_cur), then the header
 * write of update_checksum / finalize_checksum (src/cio_file.c:111, 116-124).
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <pthread.h>
#include <arpa/inet.h>

#include <crc32/crc32.h>
#include "chunkio_amd/cio_crc32_gpu.h"
#include "chunkio_amd/cio_verify.h"
#include "chunkio_amd/cio_sync.h"
#include "cio_layout.h"
#include "crc32_host.h"

/* One batch: the ranges (prepare), the routed CRC pass (run, on the calling
 * thread or on the job's own thread) and the header writes (commit). */
struct cio_sync_job {
    cio_sync_item *items;
    size_t n, m;
    int flags;
    const void **bufs;
    size_t *lens, *idx;
    uint32_t *seeds, *raw;
    int devs[64];
    int ndev;
    int rc;          /* prepare / run result */
    int threaded;
    pthread_t th;
    cioa_route_plan plan;       /* engines of the CRC pass, decided before it starts */
    /* what a threaded pass leaves in its thread's locals, handed to the
     * caller's thread by end(): cio_gpu_last_error(), cio_gpu_pipe_last_timing() */
    char err[512];
    double timing[6];
    int have_timing;
};

static void job_free(cio_sync_job *j)
{
    free(j->bufs);
    free(j->lens);
    free(j->idx);
    free(j->seeds);
    free(j->raw);
    free(j);
}

static int job_prepare(cio_sync_job *j)
{
    const size_t n = j->n;
    j->bufs = malloc(n * sizeof(*j->bufs));
    j->lens = malloc(n * sizeof(*j->lens));
    j->idx = malloc(n * sizeof(*j->idx));
    j->seeds = malloc(n * sizeof(*j->seeds));
    j->raw = malloc(n * sizeof(*j->raw));
    if (!j->bufs || !j->lens || !j->idx || !j->seeds || !j->raw) {
        return CIO_ERROR;
    }
    for (size_t i = 0; i < n; i++) {
        cio_sync_item *it = &j->items[i];
        it->status = CIO_OK;
        if (!it->map || it->fs_size < CIOA_HDR_MIN || it->map[0] != CIOA_HDR_ID_00 ||
            it->map[1] != CIOA_HDR_ID_01) {
            it->status = CIO_CORRUPTED;
            continue;
        }
        const uint64_t clen = cioa_st_get_content_len_field(it->map);
        const uint64_t meta = cioa_st_meta_len(it->map);
        const uint64_t end = it->data_end ? it->data_end : CIOA_HDR_MIN + meta + clen;
        if (end > it->fs_size || it->crc_end < CIOA_HDR_CONTENT_OFFSET || it->crc_end > end) {
            it->status = CIO_CORRUPTED;
            continue;
        }
        j->bufs[j->m] = it->map + it->crc_end;
        j->lens[j->m] = (size_t) (end - it->crc_end);
        j->seeds[j->m] = it->crc_cur;
        j->idx[j->m] = i;
        it->crc_end = end;      /* committed in job_commit, after the batch ran */
        j->m++;
    }
    return CIO_OK;
}

static void *job_run(void *arg)
{
    cio_sync_job *j = (cio_sync_job *) arg;
    j->rc = cioa_crc_batch_route_planned(j->bufs, j->lens, j->seeds, j->raw, j->m, j->ndev > 0 ? j->devs : NULL,
                                         j->ndev, &j->plan);
    if (j->threaded) {
        if (j->rc != CIO_OK) {
            snprintf(j->err, sizeof(j->err), "%s", cio_gpu_last_error());
        }
        else if (j->plan.k > 0) {
            j->have_timing = cio_gpu_pipe_last_timing(j->timing, 6) == CIO_OK;
        }
    }
    return NULL;
}

static int job_commit(cio_sync_job *j)
{
    if (j->rc != CIO_OK) {
        /* restore the ranges: nothing was written */
        for (size_t k = 0; k < j->m; k++) {
            cio_sync_item *it = &j->items[j->idx[k]];
            it->crc_end = (uint64_t) ((const unsigned char *) j->bufs[k] - it->map);
        }
        return CIO_ERROR;
    }
    for (size_t k = 0; k < j->m; k++) {
        cio_sync_item *it = &j->items[j->idx[k]];
        it->crc_cur = j->raw[k];
        crc_t v;
        if (j->flags & CIOA_SYNC_FINALIZE) {
            v = htonl((uint32_t) crc_finalize((crc_t) j->raw[k]));   /* finalize_checksum */
        } else {
            v = (crc_t) j->raw[k];                                   /* update_checksum :111 */
        }
        memcpy(it->map + 2, &v, sizeof(v));
        /* cio_file_native_sync (src/cio_file_unix.c:477-497): MS_SYNC under
         * CIO_FULL_SYNC, else MS_ASYNC; a failed msync fails the sync
         * (cio_file.c:1231-1236), the chunk stays unsynced. */
        if ((j->flags & (CIOA_SYNC_MSYNC | CIOA_SYNC_FULL)) &&
            msync(it->map, it->fs_size, (j->flags & CIOA_SYNC_FULL) ? MS_SYNC : MS_ASYNC) != 0) {
            it->status = CIO_ERROR;
        }
    }
    return CIO_OK;
}

static int job_start(cio_sync_item *items, size_t n, int flags, const int *devices, int ndev, int async,
                     cio_sync_job **out)
{
    *out = NULL;
    if (n > 0 && !items) {
        return CIO_ERROR;
    }
    cio_sync_job *j = calloc(1, sizeof(*j));
    if (!j) {
        return CIO_ERROR;
    }
    j->items = items;
    j->n = n;
    j->flags = flags;
    if (n > 0 && (j->rc = job_prepare(j)) != CIO_OK) {
        job_free(j);
        return CIO_ERROR;
    }
    if (devices && ndev > 0) {
        j->ndev = ndev < 64 ? ndev : 64;
        memcpy(j->devs, devices, (size_t) j->ndev * sizeof(int));
    }
    if (j->m > 0) {
        cioa_crc_route_plan(j->lens, j->m, j->ndev > 0 ? j->devs : NULL, j->ndev, 0, &j->plan);
    }
    /* A pass on its own thread that will use a GPU runs on the caller's
     * current device (a new thread starts on device 0).  A host-only pass
     * never asks: it must not start the HIP runtime. */
    if (async && j->m > 0 && j->plan.k > 0 && j->ndev == 0) {
        cioa_note_hip_probe();
        const int cur = cio_gpu_get_device();
        if (cur >= 0) {
            j->devs[0] = cur;
            j->ndev = 1;
        }
    }
    if (j->m > 0) {
        j->threaded = async;
        if (!async || pthread_create(&j->th, NULL, job_run, j) != 0) {
            j->threaded = 0;
            job_run(j);
        }
    }
    *out = j;
    return CIO_OK;
}

/* begin() with the CRC pass on the calling thread (async = 0): the chunk
 * layer's synchronous sync goes through the same job without a thread. */
int cioa_file_sync_batch_start(cio_sync_item *items, size_t n, int flags, const int *devices, int ndev, int async,
                               cio_sync_job **job)
{
    if (!job) {
        return CIO_ERROR;
    }
    return job_start(items, n, flags, devices, ndev, async, job);
}

int cio_file_sync_batch_begin(cio_sync_item *items, size_t n, int flags, const int *devices, int ndev,
                              cio_sync_job **job)
{
    if (!job) {
        return CIO_ERROR;
    }
    return job_start(items, n, flags, devices, ndev, 1, job);
}

int cio_file_sync_batch_end(cio_sync_job *job)
{
    if (!job) {
        return CIO_ERROR;
    }
    if (job->threaded) {
        pthread_join(job->th, NULL);
        if (job->rc != CIO_OK && job->err[0]) {
            (void) cioa_fail_msg(job->err, NULL);
        }
        if (job->have_timing) {
            cioa_pipe_timing_set(job->timing);
        }
    }
    const int rc = job->m > 0 ? job_commit(job) : CIO_OK;
    job_free(job);
    return rc;
}

int cio_file_sync_batch_multi(cio_sync_item *items, size_t n, int flags, const int *devices, int ndev)
{
    if (n == 0) {
        return CIO_OK;
    }
    cio_sync_job *j;
    if (job_start(items, n, flags, devices, ndev, 0, &j) != CIO_OK) {
        return CIO_ERROR;
    }
    return cio_file_sync_batch_end(j);
}

int cio_file_sync_batch(cio_sync_item *items, size_t n, int flags)
{
    return cio_file_sync_batch_multi(items, n, flags, NULL, 0);
}
