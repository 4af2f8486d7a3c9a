/*
 * cio_verify.h -- batched verify-on-load of chunkio chunk files.
 *
 * chunkio verifies a chunk when it maps an existing file: cio_scan_stream_files
 * (src/cio_scan.c:105) -> cio_chunk_open -> cio_file_open -> mmap_file
 * (src/cio_file.c:345-493) -> cio_file_format_check (src/cio_file.c:187-294).
 * One chunk at a time, single-threaded.  cio_file_verify_batch() runs the same
 * checks over N mapped chunk files and computes all their CRCs in ONE batch
 * -- on the GPU (cio_crc32_batch_host_multi), or on the host's crc_update
 * when the batch routes there (cio_crc32_cpu_max(): small batches, or any
 * batch when host CRC threads are granted, cio_crc32_gpu.h) -- returning per
 * chunk exactly what the reference would have recorded:
 *
 *   magic bytes C1 00                        else CIO_ERR_BAD_LAYOUT     (cio_file.c:230-236)
 *   content length (BE u32 @10), legacy       else CIO_ERR_BAD_FILE_SIZE  (cio_file_st.h:129-179,
 *     inference when the field is 0                                       cio_file.c:243-251)
 *   24 + meta_len + content_len <= fs_size    else CIO_ERR_BAD_FILE_SIZE  (cio_file.c:254-264)
 *   8-byte memcmp of map+2 against htonl(crc_finalize(crc)) held in an
 *   8-byte crc_t                              else CIO_ERR_BAD_CHECKSUM   (cio_file.c:266-290)
 *
 * status is CIO_OK or CIO_CORRUPTED (chunkio.h:50-53); error is one of the
 * CIO_ERR_* codes (cio_error.h:29-32) or 0.  On success crc_raw is the
 * un-finalized CRC the reference keeps in cf->crc_cur for later appends.
 *
 * It is also the file-level half of a batched cio_chunk_up (cio_file_up,
 * cio_file.c:816-883, over many down chunks): map the chunks within the
 * max_chunks_up budget, verify them in one call, count the ones that passed,
 * and go on with the slots the failures freed -- INTEGRATION.md's sketch, and
 * what cioa_chunk_up_batch (cioa_chunk.h) does in this repo's chunk layer.
 */
#ifndef CIO_VERIFY_H
#define CIO_VERIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef CIO_CORRUPTED
#define CIO_CORRUPTED          -3
#endif
#ifndef CIO_ERR_BAD_CHECKSUM
#define CIO_ERR_BAD_CHECKSUM  -10
#define CIO_ERR_BAD_LAYOUT    -11
#define CIO_ERR_PERMISSION    -12
#define CIO_ERR_BAD_FILE_SIZE -13
#endif

/* flags */
#define CIOA_VERIFY_CHECKSUM   4   /* same value as CIO_CHECKSUM (chunkio.h:44) */
#define CIOA_VERIFY_DELETE_IRRECOVERABLE 16
                                   /* same value as CIO_DELETE_IRRECOVERABLE (chunkio.h:46):
                                      cio_verify_paths* unlink every file that failed as
                                      CIO_CORRUPTED with BAD_CHECKSUM / BAD_FILE_SIZE /
                                      BAD_LAYOUT (src/cio_scan.c:107-118) */
#define CIOA_VERIFY_WRITEBACK  64  /* the maps are writable (chunkio's CIO_OPEN_RW):
                                      an inferred legacy content length is written
                                      back, and an empty file is initialised (init
                                      header, crc_raw 0xBE26ED00) instead of failing
                                      with CIO_ERR_PERMISSION (cio_file.c:388-393) */

typedef struct cio_verify_item {
    /* inputs */
    unsigned char *map;     /* mapped chunk file, fs_size bytes readable (for an
                               empty file opened RW: >= 24 writable bytes) */
    size_t fs_size;         /* file size (fstat) */
    int taint;              /* cf->taint_flag; 0 for a freshly opened file */
    /* outputs */
    int status;             /* CIO_OK, CIO_CORRUPTED, or CIO_ERROR (no map) */
    int error;              /* 0 or CIO_ERR_BAD_LAYOUT / _BAD_FILE_SIZE / _BAD_CHECKSUM /
                               _PERMISSION */
    uint32_t crc_raw;       /* un-finalized CRC of [map+22, 24+meta_len+content_len) */
    uint16_t meta_len;
    uint64_t content_len;   /* cf->data_size */
} cio_verify_item;

/* Verify n mapped chunk images.  Returns CIO_OK if the batch ran (individual
 * chunks may still be CIO_CORRUPTED), CIO_ERROR on a GPU/library failure.
 * Runs on the calling thread's current device. */
int cio_file_verify_batch(cio_verify_item *items, size_t n, int flags);

/* The same with the CRC pass spread over GPUs (chunk k of the checked ones ->
 * devices[k % ndev], cio_crc32_batch_host_multi); ndev <= 0: current device. */
int cio_file_verify_batch_multi(cio_verify_item *items, size_t n, int flags,
                                const int *devices, int ndev);

/* Open (read-only unless CIOA_VERIFY_WRITEBACK) + verify n chunk files, the
 * batched equivalent of loading a stream directory
 * (cio_scan_stream_files, src/cio_scan.c:39-125).  status[i], error[i],
 * crc_raw[i] per file; a file that cannot be opened, stat'ed or read gets
 * CIO_ERROR.  The files are not mapped: headers are read with pread() on up
 * to 16 host threads, and the CRC regions stream from the files into the GPU
 * pipeline (cio_crc32_batch_fd_multi: pread through a per-thread bounce
 * buffer, streaming stores into pinned staging).  With CIOA_VERIFY_WRITEBACK the files
 * are opened read-write (inferred legacy lengths written back, empty files
 * initialised and, since this call also closes them, left as the reference's
 * close leaves them: synced, with htonl(crc_finalize(0xBE26ED00)) =
 * 41 d9 12 ff in the CRC field when checksums are on, so the next verify
 * passes).  With CIOA_VERIFY_DELETE_IRRECOVERABLE the irrecoverable
 * files are unlinked after the batch, as cio_scan does. */
int cio_verify_paths(const char *const *paths, size_t n, int flags, int *status,
                     int *error, uint32_t *crc_raw);

/* cio_verify_paths with the CRC pass spread over GPUs (as above). */
int cio_verify_paths_multi(const char *const *paths, size_t n, int flags,
                           const int *devices, int ndev, int *status,
                           int *error, uint32_t *crc_raw);

#ifdef __cplusplus
}
#endif

#endif /* CIO_VERIFY_H */
