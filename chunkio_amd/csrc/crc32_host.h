/* Internal host-side declarations shared by the C and HIP translation units. */
#ifndef CIOA_CRC32_HOST_H
#define CIOA_CRC32_HOST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CIOA_POLY 0xEDB88320u

uint64_t cioa_crc_update_host(uint64_t crc, const void *data, size_t len);
const uint32_t *cioa_byte_table(void);
uint32_t cioa_multmodp(uint32_t a, uint32_t b);
uint32_t cioa_xpow8n(uint64_t n);
void cioa_gen_slice4(uint32_t out[4][256]);
void cioa_gen_shift_table(uint32_t out[4][256], uint64_t dist);
void cioa_gen_xpow8_table(uint32_t *out, size_t count, uint64_t unit_bytes);

/* Copy into pinned staging (non-temporal stores where the CPU has AVX2);
 * cioa_stage_fence() before publishing the copied bytes to another thread. */
void cioa_stage_copy(void *dst, const void *src, size_t n);
int cioa_stage_nt(void);            /* 1 when cioa_stage_copy uses streaming stores */
void cioa_stage_fence(void);

/* getenv(name) for a diagnostic / A/B switch (kernel choice, lane layout,
 * grid, read-stream probes, host-path pins, staging sizes): honoured only
 * when CIO_GPU_DIAG=1 is also set, else NULL, so a stray variable in a
 * deployment cannot change the path.  INTEGRATION.md lists them. */
const char *cioa_diag_getenv(const char *name);

/* Record an error message for cio_gpu_last_error(); returns CIO_ERROR (-1). */
int cioa_fail_msg(const char *what, const char *detail);

/* crc_route.c: the chunk layer's CRCs over host memory / file ranges -- the
 * host crc_update when the batch totals at most cio_crc32_cpu_max() bytes,
 * else the GPU batch (cio_crc32_batch_host_multi / _fd_multi). */
int cioa_crc_batch_route(const void *const *bufs, const size_t *lens, const uint32_t *seeds, uint32_t *out_raw,
                         size_t n, const int *devices, int ndev);
/* Counts a query of the HIP runtime made on the route's behalf (test hook). */
void cioa_note_hip_probe(void);

/* The same in two steps: which engine(s) a batch will use (k chunks on the
 * GPU: 0 = the host alone, n = the GPU alone, else a split), then the run.
 * Planning never touches HIP unless a split could happen (it then checks that
 * a GPU exists), so a caller can decide on GPU set-up before running. */
typedef struct cioa_route_plan {
    size_t k;
    int gpu_bound;
} cioa_route_plan;
void cioa_crc_route_plan(const size_t *lens, size_t n, const int *devices, int ndev, int fd, cioa_route_plan *plan);
int cioa_crc_batch_route_planned(const void *const *bufs, const size_t *lens, const uint32_t *seeds,
                                 uint32_t *out_raw, size_t n, const int *devices, int ndev,
                                 const cioa_route_plan *plan);
int cioa_crc_fd_route(const int *fds, const uint64_t *foffs, const size_t *lens, const uint32_t *seeds,
                      uint32_t *out_raw, size_t n, const int *devices, int ndev);

/* cio_sync.c: cio_file_sync_batch_begin with the CRC pass on a thread of its
 * own (async = 1) or on the calling thread (async = 0); end() as usual. */
struct cio_sync_item;
struct cio_sync_job;
int cioa_file_sync_batch_start(struct cio_sync_item *items, size_t n, int flags, const int *devices, int ndev,
                               int async, struct cio_sync_job **job);

/* host_pipeline.hip: set the calling thread's cio_gpu_pipe_last_timing record
 * (6 values, as that call returns them). */
void cioa_pipe_timing_set(const double *v);

uint32_t cio_crc32_shift(uint32_t raw_state, uint64_t nbytes);
uint32_t cio_crc32_combine(uint32_t raw_a, uint32_t raw0_b, uint64_t len_b);

#ifdef __cplusplus
}
#endif

#endif
