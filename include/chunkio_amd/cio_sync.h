/*
 * cio_sync.h -- batched sync of chunk files whose appends deferred the CRC.
 *
 * In chunkio every cio_file_write runs crc_update over the caller's buffer
 * before copying it (update_checksum, src/cio_file.c:97-113, called at :1058)
 * and stores the raw 8-byte state at map+2 (:111); cio_file_sync finalizes
 * it (finalize_checksum, :116-124, called at :1227-1229).  The CPU CRC is on
 * every append's critical path.
 *
 * With the CRC deferred, appends only copy; cio_file_sync_batch() then brings
 * N dirty chunks up to date in ONE batch: for each chunk the bytes
 * [crc_end, 24 + meta_len + content_len) not yet covered are CRC'd with
 * crc_cur as the seed (crc_update(crc_cur, ...)) on the GPU
 * (cio_crc32_batch_host_multi) or, when the batch routes to the host
 * (cio_crc32_cpu_max(), cio_crc32_gpu.h), on the host's crc_update; and the
 * header is written exactly as the reference would have left it:
 *
 *   CIOA_SYNC_FINALIZE: htonl(crc_finalize(crc)) in an 8-byte crc_t at map+2
 *                       (bytes 2..5 = big-endian CRC, 6..9 = 0), cio_file.c:116-124
 *   otherwise:          the raw 8-byte crc_t state at map+2, cio_file.c:111
 *
 * The resulting file bytes are identical to the reference's write/sync
 * sequence.  A write_at (crc_reset, src/cio_chunk.c:199-201) or a metadata
 * move (adjust_layout, src/cio_file.c:130-146) is expressed by the caller as
 * crc_end = 22, crc_cur = 0xFFFFFFFF (a full recompute from crc_init()).
 */
#ifndef CIO_SYNC_H
#define CIO_SYNC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CIOA_SYNC_FINALIZE  1   /* write the finalized CRC (cio_file_sync) */
#define CIOA_SYNC_MSYNC     2   /* msync(MS_ASYNC) each map after the header write (cio_file.c:1232) */
#define CIOA_SYNC_FULL      8   /* msync(MS_SYNC) instead: chunkio's CIO_FULL_SYNC (chunkio.h:45,
                                   cio_file_unix.c:481-486); same value as that flag */

typedef struct cio_sync_item {
    unsigned char *map;   /* writable mapped chunk file: magic C1 00, meta_len (BE u16 @22),
                             content_len (BE u32 @10) valid */
    size_t fs_size;       /* mapped size */
    uint64_t crc_end;     /* in/out: file offset up to which crc_cur is current (>= 22) */
    uint32_t crc_cur;     /* in/out: raw CRC state over [22, crc_end) (cf->crc_cur) */
    int status;           /* out: CIO_OK, CIO_CORRUPTED for a bad header / range, or CIO_ERROR
                             when msync failed (header written, chunk not durable: the
                             caller keeps it unsynced, as cio_file_sync does on that error) */
    uint64_t data_end;    /* in: end of the CRC region, 24 + meta_len + cf->data_size, or 0 to
                             take it from the header's content length.  They differ after a
                             transaction rollback (src/cio_chunk.c:476-502 restores data_size
                             but not the header field) */
} cio_sync_item;

/* Bring n chunks' CRCs up to date in one GPU batch and write their headers.
 * Returns CIO_OK if the batch ran (items may still be CIO_CORRUPTED),
 * CIO_ERROR on a GPU/library failure (then no header was written). */
int cio_file_sync_batch(cio_sync_item *items, size_t n, int flags);

/* The same with the CRC pass spread over GPUs (cio_crc32_batch_host_multi:
 * chunk k -> devices[k % ndev]); ndev <= 0: the current device. */
int cio_file_sync_batch_multi(cio_sync_item *items, size_t n, int flags,
                              const int *devices, int ndev);

/* The same batch with the CRC pass on a thread of its own, so the caller can
 * go on (e.g. write the next chunks) while it runs.  begin() checks the
 * headers and starts the pass (on the devices given, else the caller's
 * current device); end() waits for it, writes the headers, runs the msyncs and
 * frees the job.  Between the two the items and the mapped bytes they cover
 * must stay as they are.  begin() returns CIO_ERROR with *job = NULL only when
 * nothing started (no memory); end() returns what cio_file_sync_batch_multi
 * returns.  Every job begun must be ended. */
typedef struct cio_sync_job cio_sync_job;
int cio_file_sync_batch_begin(cio_sync_item *items, size_t n, int flags,
                              const int *devices, int ndev, cio_sync_job **job);
int cio_file_sync_batch_end(cio_sync_job *job);

#ifdef __cplusplus
}
#endif

#endif /* CIO_SYNC_H */
