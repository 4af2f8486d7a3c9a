/*
 * cioa_chunk.h -- chunkio's filesystem chunk API (write / write_at / metadata /
 * sync / up / down / transactions / scan), in C, with the CRC-32 lifecycle
 * driven by the batched GPU path of libchunkio_amd.so.
 *
 * Every function mirrors the reference function of the same name without
 * the "a" (cioa_chunk_write <-> cio_chunk_write, ...): same arguments, same
 * return values (CIO_OK 0 / CIO_ERROR -1 / CIO_RETRY -2 / CIO_CORRUPTED -3),
 * same error numbers in cioa_error_get(), and byte-identical chunk files.
 * The prefix keeps both libraries linkable into one process.
 *
 *   cioa_create / cioa_destroy          src/chunkio.c:84-207 (cio_create), cio_destroy
 *   cioa_set_max_chunks_up              src/chunkio.c:331-339
 *   cioa_set_realloc_size_hint          src/chunkio.c:341-359
 *   cioa_stream_create                  src/cio_stream.c:113-178
 *   cioa_stream_size_chunks_up          src/cio_stream.c:258-276
 *   cioa_chunk_open / _close / _delete  src/cio_chunk.c:30-178 -> src/cio_file.c:636-810, 961-991
 *   cioa_chunk_write / _write_at        src/cio_chunk.c:184-227 -> cio_file.c:994-1073
 *   cioa_chunk_sync                     src/cio_chunk.c:229-242 -> cio_file.c:1147-1250
 *                                       (CIO_TRIM_FILES :1192-1224, CIO_FULL_SYNC msync)
 *   cioa_chunk_get_content[_copy]       src/cio_chunk.c:244-291, cio_file.c:505-558
 *   cioa_chunk_get_content_size / _real_size / _hash   src/cio_chunk.c:315-382
 *   cioa_chunk_lock / _unlock / _is_locked             src/cio_chunk.c:384-416
 *   cioa_chunk_tx_begin / _commit / _rollback          src/cio_chunk.c:423-502
 *   cioa_chunk_is_up / _up / _up_force / _down         src/cio_chunk.c:509-605, cio_file.c:816-959
 *   cioa_chunk_up_batch / _up_force_batch  the same up over many chunks, verifies batched
 *   cioa_meta_write / _read / _cmp / _size             src/cio_meta.c:46-180, cio_file.c:1075-1145
 *   cioa_scan_dump                      src/cio_scan.c:171-190, cio_file.c:1316-1375 (tools/cio -l)
 *   cioa_scan_stream                    src/cio_scan.c:39-125 (verify-on-load of a stream
 *                                       directory, CIO_DELETE_IRRECOVERABLE :107-118)
 *   cioa_scan_streams                   src/cio_scan.c:128-162 (every stream of the root)
 *
 * Where the CRC runs:
 *   - verify on open/up/scan (cio_file_format_check, cio_file.c:266-290): the
 *     batched verify (cio_file_verify_batch_multi, routed by crc_route.c to
 *     the GPU or, for small batches, the host crc_update); cioa_scan_stream
 *     and cioa_scan_streams verify every chunk they map in ONE batch (across
 *     streams), and cioa_chunk_up_batch the chunks it brings up;
 *   - the per-write update (update_checksum, cio_file.c:97-113): crc_update
 *     on the caller's buffer, as the reference does -- unless the context
 *     has CIOA_DEFERRED_CRC, where writes only copy and the CRC of every
 *     byte not yet covered is computed at sync time (routed the same way),
 *     for many chunks at once with cioa_chunk_sync_batch
 *     (cio_file_sync_batch_multi);
 *   - full recomputes (write_at, metadata rewrite: cio_file.c:103-108,
 *     136-140): one routed batch (immediate mode) or folded into the next
 *     sync (deferred mode).
 * Either way the files are byte-identical to the reference's after a sync.
 *
 * Not thread-safe per context, like the reference: one context per thread.
 * GPU work runs on the context's devices (cioa_set_devices), default the
 * calling thread's current device.
 */
#ifndef CIOA_CHUNK_H
#define CIOA_CHUNK_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <sys/types.h>

#ifdef __cplusplus
extern "C" {
#endif

/* flags: chunkio.h:40-47 values */
#ifndef CIO_OPEN
#define CIO_OPEN                 1
#define CIO_OPEN_RW              CIO_OPEN
#define CIO_OPEN_RD              2
#define CIO_CHECKSUM             4
#define CIO_FULL_SYNC            8
#define CIO_DELETE_IRRECOVERABLE 16
#define CIO_TRIM_FILES           32
#endif
#define CIOA_DEFERRED_CRC        128   /* appends only copy; CRC at sync, in routed batches */

#ifndef CIO_OK
#define CIO_OK       0
#define CIO_ERROR   -1
#endif
#ifndef CIO_RETRY
#define CIO_RETRY   -2
#endif
#ifndef CIO_CORRUPTED
#define CIO_CORRUPTED -3
#endif
#ifndef CIO_ERR_BAD_CHECKSUM
#define CIO_ERR_BAD_CHECKSUM  -10
#define CIO_ERR_BAD_LAYOUT    -11
#define CIO_ERR_PERMISSION    -12
#define CIO_ERR_BAD_FILE_SIZE -13
#endif

#define CIOA_MAX_CHUNKS_UP 64          /* CIO_MAX_CHUNKS_UP, chunkio.h:63 */

typedef struct cioa_ctx cioa_ctx;
typedef struct cioa_stream cioa_stream;
typedef struct cioa_chunk cioa_chunk;

/* ---- context ------------------------------------------------------------ */

/* root_path is created if missing.  flags: CIO_OPEN_RW/RD (RW if neither),
 * CIO_CHECKSUM, CIO_FULL_SYNC, CIO_DELETE_IRRECOVERABLE, CIO_TRIM_FILES,
 * CIOA_DEFERRED_CRC. */
cioa_ctx *cioa_create(const char *root_path, int flags);
void cioa_destroy(cioa_ctx *ctx);              /* closes (and syncs) every chunk */
int  cioa_set_max_chunks_up(cioa_ctx *ctx, int n);
int  cioa_set_realloc_size_hint(cioa_ctx *ctx, size_t realloc_size_hint);
void cioa_enable_file_trimming(cioa_ctx *ctx);
void cioa_disable_file_trimming(cioa_ctx *ctx);
int  cioa_get_flags(const cioa_ctx *ctx);
/* GPUs for the context's batched CRC passes (chunk k -> devices[k % n]);
 * n <= 0: the calling thread's current device. */
int  cioa_set_devices(cioa_ctx *ctx, const int *devices, int n);
int  cioa_last_chunk_error(const cioa_ctx *ctx);
size_t cioa_total_chunks(const cioa_ctx *ctx);
size_t cioa_total_chunks_up(const cioa_ctx *ctx);

/* ---- streams ------------------------------------------------------------ */

cioa_stream *cioa_stream_create(cioa_ctx *ctx, const char *name);
cioa_stream *cioa_stream_get(cioa_ctx *ctx, const char *name);
size_t cioa_stream_size_chunks_up(cioa_stream *st);
/* Chunks of a stream in open order: fills up to cap, returns the count. */
size_t cioa_stream_chunks(cioa_stream *st, cioa_chunk **out, size_t cap);

/* Verify-on-load of root_path/<stream> (cio_scan_stream_files): every
 * regular file not starting with '.' (and ending in chunk_extension if
 * given) becomes a chunk, in name order.  Up to the free max_chunks_up
 * slots they are opened, mapped and verified in ONE batched GPU pass; as in
 * the reference a chunk takes a slot only once it passed (cio_file.c:490),
 * so when some fail, the freed slots go to the next files in another batch.
 * The rest are registered down (unverified, as the reference leaves them).
 * A chunk that fails its load is not registered; with
 * CIO_DELETE_IRRECOVERABLE the file is deleted when the failure was
 * BAD_CHECKSUM / BAD_FILE_SIZE / BAD_LAYOUT.  If a batch cannot run at all
 * (GPU failure), its chunks are registered down, unverified (a later
 * cioa_chunk_up verifies them), and cioa_last_chunk_error() returns
 * CIO_ERROR afterwards (cio_gpu_last_error() has the reason).  Returns the
 * stream (created if needed) or NULL. */
cioa_stream *cioa_scan_stream(cioa_ctx *ctx, const char *stream, const char *chunk_extension);
/* cio_scan_streams (src/cio_scan.c:128-162, what cio_load runs): every
 * directory under the root (names starting with '.' skipped, name order) is a
 * stream loaded as cioa_scan_stream loads one, with the same result as
 * loading them one after the other -- but every stream's files go through
 * one set of rounds, so a round's verify batch spans streams (a root of many
 * small streams fills one GPU batch).  0, or -1 when the root cannot be read. */
int cioa_scan_streams(cioa_ctx *ctx, const char *chunk_extension);

/* The listing of `tools/cio -l` (cio_scan_dump, src/cio_scan.c:171-190 ->
 * cio_file_scan_dump, src/cio_file.c:1316-1375), same text, to out: per stream
 * " stream:%-60s%i chunks", per chunk "        %-60s" then, with CIO_CHECKSUM and a
 * mismatch, "checksum error=%08x expected=%08x, " (header value first, as the
 * reference prints them), then "meta_len=%d, data_size=%zu, crc=%08x".  Down
 * chunks are brought up for it and down again; one that cannot come up is left
 * out.  The recompute is the reference's: crc_update(crc_cur, region) --
 * seeded from crc_cur, not crc_init(), so a chunk loaded with a verified
 * crc_cur lists as a checksum error, as it does in the reference.
 * A stream's recomputes run as one GPU batch. */
int cioa_scan_dump(cioa_ctx *ctx, FILE *out);

/* ---- chunks ------------------------------------------------------------- */

cioa_chunk *cioa_chunk_open(cioa_ctx *ctx, cioa_stream *st, const char *name, int flags,
                            size_t size, int *err);
void cioa_chunk_close(cioa_chunk *ch, int delete_file);
int  cioa_chunk_delete(cioa_ctx *ctx, cioa_stream *st, const char *name);
int  cioa_chunk_write(cioa_chunk *ch, const void *buf, size_t count);
int  cioa_chunk_write_at(cioa_chunk *ch, off_t offset, const void *buf, size_t count);
int  cioa_chunk_sync(cioa_chunk *ch);
/* Sync n chunks: trims and header finalisation as cioa_chunk_sync, with the
 * deferred CRCs of all of them in ONE GPU pass.  CIO_OK when every chunk
 * synced; otherwise CIO_ERROR (chunks that failed stay unsynced). */
int  cioa_chunk_sync_batch(cioa_chunk **chunks, size_t n);
/* The same in two halves, so the caller can go on while the CRC pass runs on
 * a thread of its own (cio_file_sync_batch_begin/end): begin() syncs the
 * chunks that need no CRC pass and starts the pass over the deferred ones;
 * end() waits for it, writes the finalized headers, msyncs and marks the
 * chunks synced, returns what cioa_chunk_sync_batch would have and frees the
 * job.  Until then a chunk of the batch is held: writing, syncing, a metadata
 * write, a transaction, down or close of it finishes the whole batch first
 * (the job stays valid for end()).  begin() fails (*job = NULL) only without
 * memory; every job begun must be ended (also after its context is gone). */
typedef struct cioa_sync_job cioa_sync_job;
int  cioa_chunk_sync_batch_begin(cioa_chunk **chunks, size_t n, cioa_sync_job **job);
int  cioa_chunk_sync_batch_end(cioa_sync_job *job);
int  cioa_chunk_get_content(cioa_chunk *ch, char **buf, size_t *size);
int  cioa_chunk_get_content_copy(cioa_chunk *ch, void **out_buf, size_t *out_size);
ssize_t cioa_chunk_get_content_size(cioa_chunk *ch);
size_t  cioa_chunk_get_content_end_pos(cioa_chunk *ch);   /* address past the content; 0 when down */
int  cioa_chunk_is_file(cioa_chunk *ch);                  /* 1: every chunk here is file-backed */
void cioa_chunk_close_stream(cioa_stream *st);            /* close every chunk, files kept */
ssize_t cioa_chunk_get_real_size(cioa_chunk *ch);
char *cioa_chunk_hash(cioa_chunk *ch);        /* map + 2, NULL when down */
int  cioa_chunk_lock(cioa_chunk *ch);
int  cioa_chunk_unlock(cioa_chunk *ch);
int  cioa_chunk_is_locked(cioa_chunk *ch);
int  cioa_chunk_tx_begin(cioa_chunk *ch);
int  cioa_chunk_tx_commit(cioa_chunk *ch);
int  cioa_chunk_tx_rollback(cioa_chunk *ch);
int  cioa_chunk_is_up(cioa_chunk *ch);
int  cioa_chunk_up(cioa_chunk *ch);
int  cioa_chunk_up_force(cioa_chunk *ch);
/* cio_chunk_up / cio_chunk_up_force (src/cio_chunk.c:573-605 -> cio_file_up,
 * cio_file.c:816-883) over n chunks with the outcome of n calls in list
 * order -- per-chunk status[i] (CIO_OK / CIO_ERROR / CIO_CORRUPTED /
 * CIO_RETRY, may be NULL), error numbers, crc_cur, the max_chunks_up budget
 * (enforced: a chunk that fails its check frees its slot for the next) --
 * with the CRC verifies of the chunks brought up in as few routed batches as
 * that order allows (one, unless failures free slots, or the list mixes
 * contexts or open modes).  Returns CIO_OK when every chunk came up. */
int  cioa_chunk_up_batch(cioa_chunk **chunks, size_t n, int *status);
int  cioa_chunk_up_force_batch(cioa_chunk **chunks, size_t n, int *status);
int  cioa_chunk_down(cioa_chunk *ch);
const char *cioa_chunk_name(cioa_chunk *ch);
/* The chunk's mapping (NULL when down) and its mapped size (cf->map,
 * cf->alloc_size): for inspection of the on-disk bytes. */
unsigned char *cioa_chunk_map(cioa_chunk *ch, size_t *alloc_size);
int  cioa_error_get(cioa_chunk *ch);           /* cio_error_get: last CIO_ERR_* of the chunk */

/* The running raw CRC state (cf->crc_cur) and, for tests that inject faults
 * the way tests/fs.c:710 does (cf->crc_cur = 10), a setter. */
uint32_t cioa_chunk_crc_cur(cioa_chunk *ch);
void     cioa_chunk_set_crc_cur(cioa_chunk *ch, uint32_t crc);

int  cioa_meta_write(cioa_chunk *ch, const char *buf, size_t size);
int  cioa_meta_read(cioa_chunk *ch, char **meta_buf, int *meta_len);
int  cioa_meta_cmp(cioa_chunk *ch, const char *meta_buf, int meta_len);
int  cioa_meta_size(cioa_chunk *ch);

/* ---- benchmark driver ----------------------------------------------------
 * BASELINE config 1's loop (tools/cio.c:367-466, cb_cmd_perf) through this
 * API: stream "test-perf" under root, `files` chunks perf-test-NNNN.txt, each
 * opened, written `writes` times with data, synced and closed.  With
 * CIOA_DEFERRED_CRC in flags, chunks are synced `batch` at a time through
 * cioa_chunk_sync_batch (one GPU pass per batch).  *secs = wall time of the
 * loop, *bytes = bytes written (files * writes * len). */
int cioa_bench_perf_write(const char *root, const void *data, size_t len, int files, int writes,
                          int batch, int flags, double *secs, uint64_t *bytes);
/* flags bit for cioa_bench_perf_write only (not a context flag): with
 * CIOA_DEFERRED_CRC, each batch's CRC pass runs while the next batch is
 * written (cioa_chunk_sync_batch_begin / _end), the batch before it ended and
 * closed when the next begins. */
#define CIOA_BENCH_PIPELINED_SYNC 0x10000

#ifdef __cplusplus
}
#endif

#endif /* CIOA_CHUNK_H */
