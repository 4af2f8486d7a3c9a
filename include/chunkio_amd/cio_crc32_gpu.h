/*
 * cio_crc32_gpu.h -- C ABI of libchunkio_amd.so: batched CRC-32 (and SHA-1)
 * over independent chunk content buffers on an MI355X (gfx950).
 *
 * Every entry point is plain C: pointers, sizes, and an opaque HIP stream
 * passed as void* (NULL = the legacy default stream).  No torch or HIP types
 * appear in the signatures.  Return codes follow chunkio's conventions
 * (include/chunkio/chunkio.h:50-53): CIO_OK 0 / CIO_ERROR -1; the reason of
 * the last failure on the calling thread is available from
 * cio_gpu_last_error().
 *
 * What each call replaces in the reference (fluent/chunkio):
 *
 *   crc_update()                     deps/crc32/crc32.c:337-390, reached from
 *                                    src/cio_file.c:92 and :110 (header
 *                                    <crc32/crc32.h>, shipped in include/crc32)
 *   cio_crc32_batch_dev()            N independent calls of
 *   cio_crc32_plan_create/exec()     cio_file_calculate_checksum()
 *                                    (src/cio_file.c:66-94), i.e. the loop
 *                                    cio_scan_stream_files() drives through
 *                                    cio_chunk_open -> cio_file_format_check
 *                                    (src/cio_scan.c:105, src/cio_file.c:266-290)
 *                                    for device-resident chunk contents
 *   cio_crc32_batch_host()           the same over host (e.g. mmap'd) buffers:
 *                                    pinned staging + H2D + kernel + D2H
 *   cio_crc32_shift/_combine()       no reference counterpart; folds GPU partial
 *                                    CRCs into a running cf->crc_cur
 *                                    (src/cio_file.c:97-113)
 *   cio_sha1_batch_dev()             cio_sha1_init/update/final over each chunk
 *                                    (src/cio_sha1.c:26-57)
 *   cio_sha1_update/final_batch_dev  cio_sha1_update / cio_sha1_final on a
 *                                    carried context per chunk (src/cio_sha1.c:
 *                                    31-39), incl. the pre-Final state export of
 *                                    cio_sha1_hash (:41-57)
 *
 * CRC values in and out are RAW states (not finalized), exactly what
 * crc_update() takes and returns: seed 0xffffffff (= crc_init()) gives the
 * state that crc_finalize() turns into the standard CRC-32.
 */
#ifndef CIO_CRC32_GPU_H
#define CIO_CRC32_GPU_H

#include <stddef.h>
#include <stdint.h>
#include <chunkio_amd/cio_sha1_state.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef CIO_OK
#define CIO_OK       0
#define CIO_ERROR   -1
#endif

/* ---- device / library state ------------------------------------------- */

/* Initialise the device tables on the current HIP device (idempotent, thread
 * safe).  Called implicitly by every GPU entry point. */
int cio_gpu_init(void);

/* Devices.  Every single-device entry point runs on the calling thread's
 * current HIP device; these select it without HIP headers (a chunkio process
 * drives G GPUs with one host thread per device, or through the *_multi
 * entry points below).  count: visible devices (0 if none). */
int cio_gpu_device_count(void);
int cio_gpu_set_device(int dev);
int cio_gpu_get_device(void);            /* -1 on error */

/* NUMA node the device's PCIe link attaches to (sysfs), -1 if unknown.  The
 * host pipeline's copy threads run on that node's CPUs; a caller that owns
 * the chunk buffers does best to allocate them there too. */
int cio_gpu_numa_node(int dev);

/* PCI address of device `dev` ("dddd:bb:dd.f", NUL-terminated, len >= 13):
 * lets one process per GPU show which physical device it drives. */
int cio_gpu_pci_bus_id(int dev, char *buf, int len);

/* Human-readable reason for the last CIO_ERROR on this thread ("" if none). */
const char *cio_gpu_last_error(void);

/* Library build identification (kernel variant, arch). */
const char *cio_gpu_version(void);

/* ---- CRC-32 math on the host (no device needed) ------------------------ */

/* crc_update(s, zeros(n)) computed in O(log n): multiply by x^(8n) mod P. */
uint32_t cio_crc32_shift(uint32_t raw_state, uint64_t nbytes);

/* Raw state of A||B from raw0(A) (any seed), raw0(B) (ZERO-seeded raw
 * state of B) and |B|:  crc_update(s, A||B) ==
 *     cio_crc32_combine(crc_update(s, A), crc_update(0, B), |B|). */
uint32_t cio_crc32_combine(uint32_t raw_a, uint32_t raw0_b, uint64_t len_b);

/* ---- batched CRC-32, device-resident ----------------------------------- */

/*
 * A plan fixes the geometry of a batch (n chunks at byte offsets offs[i]
 * with lengths lens[i] from one device base pointer) and uploads the work
 * partition once, on the calling thread's current device; executing it is ONE
 * kernel launch on `stream` with no host synchronisation, so it can be
 * captured in a HIP graph.
 * offs/lens are HOST arrays.  Offsets and lengths may be arbitrary (any byte
 * alignment, zero-length chunks allowed).
 */
typedef struct cio_crc32_plan cio_crc32_plan;

int  cio_crc32_plan_create(cio_crc32_plan **plan, const uint64_t *offs,
                           const uint64_t *lens, size_t n);
void cio_crc32_plan_destroy(cio_crc32_plan *plan);

/* dev_seeds: device array of n raw seeds, or NULL for crc_init() each.
 * dev_out:   device array of n raw CRC states (uint32).  */
int  cio_crc32_plan_exec(const cio_crc32_plan *plan, const void *dev_base,
                         const uint32_t *dev_seeds, uint32_t *dev_out,
                         void *stream);

/* Same as cio_crc32_plan_exec, recording HIP events (from
 * cio_gpu_event_create) on `stream` immediately before and after the main
 * CRC kernel, for roofline measurement of that kernel alone. */
int  cio_crc32_plan_exec_events(const cio_crc32_plan *plan, const void *dev_base,
                                const uint32_t *dev_seeds, uint32_t *dev_out,
                                void *stream, void *ev_piece_start,
                                void *ev_piece_stop);

/* Total content bytes the plan covers (sum of lens). */
uint64_t cio_crc32_plan_bytes(const cio_crc32_plan *plan);

/* Name of the kernel the plan launches: "crc32_stream_kernel" (general
 * batches) or "crc32_small_kernel" (every chunk within one 4 KiB wave-step). */
const char *cio_crc32_plan_kernel(const cio_crc32_plan *plan);

/* ---- several device-resident batches in flight ---------------------------
 *
 * A ring of `depth` (1..8) plans of one geometry, each with its own stream.
 * cio_crc32_ring_exec() queues one batch behind everything already queued on
 * `stream` (its inputs) but does NOT make `stream` wait for it: consecutive
 * batches run on different slots, so one batch's start overlaps the previous
 * one's tail (cfg2: 85-87% of 8 TB/s with depth 2 against 78% one batch at a
 * time).  cio_crc32_ring_join(ring, stream) makes `stream` wait for every
 * batch queued so far; read the outputs after it.  A batch's dev_out must not
 * be reused before its join.  Not thread-safe per ring. */
typedef struct cio_crc32_ring cio_crc32_ring;
int  cio_crc32_ring_create(cio_crc32_ring **ring, const uint64_t *offs, const uint64_t *lens, size_t n, int depth);
int  cio_crc32_ring_exec(cio_crc32_ring *ring, const void *dev_base, const uint32_t *dev_seeds, uint32_t *dev_out,
                         void *stream);
int  cio_crc32_ring_join(cio_crc32_ring *ring, void *stream);
void cio_crc32_ring_destroy(cio_crc32_ring *ring);

/* Workgroups one launch of the plan runs (one per CU; four per CU for long
 * mixed-size batches, whose extra workgroups queue for a free CU). */
uint32_t cio_crc32_plan_workgroups(const cio_crc32_plan *plan);

/* One-shot: plan + exec + wait + destroy. */
int  cio_crc32_batch_dev(const void *dev_base, const uint64_t *offs,
                         const uint64_t *lens, const uint32_t *dev_seeds,
                         uint32_t *dev_out, size_t n, void *stream);

/* ---- batched CRC-32 over host memory (end-to-end path) ----------------- */

/* bufs[i]/lens[i]: host buffers (e.g. mmap'd chunk files, any alignment).
 * seeds: host array or NULL.  out_raw: host array of raw states.
 * Streams the batch through pinned staging buffers with H2D copies
 * overlapped with the kernels; synchronous on return. */
int  cio_crc32_batch_host(const void *const *bufs, const size_t *lens,
                          const uint32_t *seeds, uint32_t *out_raw, size_t n);

/* The same batch spread over several GPUs: chunk i goes to
 * devices[i % ndev], one host thread + pipeline + stream per device entry, no
 * collective; results are scattered back by index.  A device may be listed
 * more than once (each entry gets its own pipeline).  ndev <= 0: the current
 * device, as cio_crc32_batch_host.  Concurrent calls are safe: pipelines are
 * pooled per device and nothing global is held while a batch runs. */
int  cio_crc32_batch_host_multi(const void *const *bufs, const size_t *lens,
                                const uint32_t *seeds, uint32_t *out_raw, size_t n,
                                const int *devices, int ndev);

/* ONE host buffer split over several GPUs (SURVEY §8(e)'s optional case):
 * its len bytes are cut into ndev pieces (4 KiB multiples), piece i CRC'd on
 * devices[i] (the first seeded with `seed`, the others from 0) through
 * cio_crc32_batch_host_multi, and the piece states joined on the host with
 * cio_crc32_combine: *out_raw = crc_update(seed, buf, len).  The only
 * combine step the path has; no collective. */
int  cio_crc32_split_host_multi(const void *buf, size_t len, uint32_t seed, uint32_t *out_raw,
                                const int *devices, int ndev);

/* The same over file ranges: chunk i is bytes [foffs[i], foffs[i] + lens[i])
 * of the open file fds[i], read by the pipeline's copy threads with pread()
 * straight into pinned staging (no mapping).  For batch verifies of chunk
 * files that are not otherwise mapped (cio_verify_paths).  CIO_ERROR if a
 * range cannot be read in full. */
int  cio_crc32_batch_fd_multi(const int *fds, const uint64_t *foffs, const size_t *lens,
                              const uint32_t *seeds, uint32_t *out_raw, size_t n,
                              const int *devices, int ndev);

/* Pin a long-lived host range in place (e.g. a chunk file's MAP_SHARED
 * mapping, cio_file_unix.c:100) so that cio_crc32_batch_host DMAs the chunks
 * inside it directly, skipping the copy into pinned staging.  A staging group
 * takes the direct path only when every one of its chunks lies inside a
 * registered range; others are staged as before, so results never depend on
 * registration.  Registration pins pages (costly: do it once per mapping,
 * not per batch).  The range is pinned portable, so every device's pipeline
 * can DMA it.  CIO_ERROR when the driver cannot pin the range or it is
 * already registered; cio_crc32_host_unregister(p) takes the start address
 * given to register and waits for batch calls in flight. */
int  cio_crc32_host_register(const void *p, size_t len);
int  cio_crc32_host_unregister(const void *p);

/* Host-side legs of a host/file batch: the calling thread's own last
 * single-device batch (cio_crc32_batch_host, or a *_multi call with one
 * device); if this thread has run none (e.g. it only made *_multi calls over
 * several devices, which run on internal threads), the last device pipeline
 * of any thread to finish -- last writer wins.  out[0..5] = total ms, copy
 * into pinned staging ms (the caller's wall time over the copy, DMA issue
 * included), slot waits ms, plan builds ms, staging groups, staged bytes.
 * Fills min(n, 6) values. */
int  cio_gpu_pipe_last_timing(double *out, int n);

/* The host pipelines' plan image caches, summed over every idle pipeline of
 * every device: {entries, bytes held, hits, misses, stores, evictions,
 * pipelines}.  Fills min(n, 7) values.  A geometry is cached on its second
 * sighting; each pipeline holds at most CIO_GPU_PLAN_CACHE entries (32) and
 * CIO_GPU_PLAN_CACHE_MB megabytes (16). */
int  cio_gpu_plan_cache_stats(uint64_t *out, int n);

/* ---- batched CRC-32 on the host CPU ------------------------------------ */

/* The same batch as cio_crc32_batch_host / _fd_multi computed on the host:
 * crc_update (the library's drop-in for deps/crc32/crc32.c:337-390) on up to
 * `threads` threads of a persistent pool (the calling thread included).
 * Chunks above 1 MiB are split into pieces and folded with
 * cio_crc32_combine, so one large chunk uses every thread; small chunks are
 * grouped.  threads <= 1 is the reference's own loop on the calling thread.
 * Results are bit-identical to the GPU batch.  One batch runs in the pool at
 * a time (concurrent callers queue). */
int  cio_crc32_batch_cpu(const void *const *bufs, const size_t *lens,
                         const uint32_t *seeds, uint32_t *out_raw, size_t n,
                         int threads);
int  cio_crc32_batch_fd_cpu(const int *fds, const uint64_t *foffs, const size_t *lens,
                            const uint32_t *seeds, uint32_t *out_raw, size_t n,
                            int threads);

/* Routing of the chunk layer's CRCs over host memory.  The verify/sync
 * batches (cio_verify.h, cio_sync.h) and the chunk API (cioa_chunk.h) compute
 * a batch whose regions total at most cio_crc32_cpu_max() bytes on the host
 * (cio_crc32_batch_cpu with cio_crc32_host_threads() threads) and larger
 * batches on the GPU (cio_crc32_batch_host_multi / _fd_multi).  Same results
 * either way.  The default threshold is a cost model with rates measured on
 * the MI355X box (crc_route.c): with the default single host thread it is
 * ~17 MB per device in the call's device list; with two or more host threads
 * the host's DRAM rate beats a PCIe link and every host-memory batch stays on
 * the CPU.  CIOA_CPU_CRC_MAX (bytes) or cio_crc32_set_cpu_max() override the
 * threshold, 0 sends everything to the GPU alone (no split); CIOA_HOST_CRC_THREADS or
 * cio_crc32_set_host_threads() (1..64) set the thread count.  The
 * cio_crc32_batch_* entry points never route. */
size_t cio_crc32_cpu_max(void);
void   cio_crc32_set_cpu_max(size_t bytes);
/* Split route (default on; CIOA_SPLIT_ROUTE=0 or set_split_route(0) turn it
 * off): a large chunk-layer batch runs on the GPU and the host at once -- the
 * GPU part (first chunks) on a helper thread, a suffix of whole chunks on the
 * caller's host CRC threads -- sized so both finish together with rates
 * learned from earlier splits (crc_route.c).  Taken when it gives the GPU at
 * least 32 MB and beats the better engine alone, both for batches the
 * threshold sends to the GPU and for batches it keeps on the host.  An
 * explicit threshold (cio_crc32_set_cpu_max / CIOA_CPU_CRC_MAX) picks one
 * engine unless set_split_route(1) was also called; 0 is always the GPU
 * alone.  set_split_route(2) forces a split of every batch of 2+ chunks
 * (tests; also CIOA_SPLIT_ROUTE=2).  split_rates: {host memory T=1, host file T=1, host memory T,
 * host file T, GPU memory, GPU file} GB/s the next split is sized with, T =
 * cio_crc32_host_threads(); split_forget drops what was learned. */
int    cio_crc32_split_route(void);
void   cio_crc32_set_split_route(int on);
void   cio_crc32_split_rates(double *out, int n);
void   cio_crc32_split_forget(void);
int    cio_crc32_host_threads(void);
void   cio_crc32_set_host_threads(int threads);
/* Drop what the two setters set (back to the environment / defaults). */
void   cio_crc32_route_reset(void);

/* ---- synthetic data (benchmarks / tests) ------------------------------- */

/* Fill dev_base + offs[i] .. + lens[i] with the deterministic generator
 *   word_k(id) = splitmix64(seed ^ (0x9E3779B97F4A7C15 * (id + 1)) + k)
 * emitted little-endian (byte t of the chunk = byte t%8 of word_{t/8}(id)),
 * id = ids[i] (host array) or i when ids is NULL.  Synchronous. */
int  cio_gpu_fill_synthetic(void *dev_base, const uint64_t *offs,
                            const uint64_t *lens, const uint64_t *ids, size_t n,
                            uint64_t seed, void *stream);

/* ---- batched SHA-1, device-resident ------------------------------------ */

/* 20-byte digests (big-endian byte order, as SHA1_Final writes them) into
 * dev_digests + 20*i.  offs/lens are HOST arrays. */
int  cio_sha1_batch_dev(const void *dev_base, const uint64_t *offs,
                        const uint64_t *lens, uint8_t *dev_digests, size_t n,
                        void *stream);

/* The same with DEVICE-resident dev_offs/dev_lens (n entries each): one kernel
 * launch on `stream`, no allocation, no host synchronisation, so it can be
 * captured in a HIP graph and repeated over a resident batch like
 * cio_crc32_plan_exec. */
int  cio_sha1_batch_dev_async(const void *dev_base, const uint64_t *dev_offs,
                              const uint64_t *dev_lens, uint8_t *dev_digests,
                              size_t n, void *stream);

/* ---- SHA-1 with continuation (SHA1_Init / SHA1_Update / SHA1_Final) ----- */

/* Per-chunk SHA-1 context: OpenSSL's SHA_CTX, byte for byte
 * (chunkio_amd/cio_sha1_state.h) -- the context cio_sha1_init/update/final
 * carry in struct cio_sha1 (src/cio_sha1.c:26-39) and cio_sha1_hash exports
 * before its SHA1_Final "for future iterations and updates" (:41-57).  A
 * context made by OpenSSL or by the host cio_sha1_* (cio_sha1.h) continues
 * here, and one continued here continues there.  96 bytes, plain data:
 * arrays of it live in device memory for the batch calls below. */

/* SHA1_Init of n states in HOST memory (copy them to the device after). */
void cio_sha1_state_init(cio_sha1_state *states, size_t n);

/* SHA1_Update of chunk i (dev_base + dev_offs[i], dev_lens[i] bytes) into
 * dev_states[i], for every i in one launch (device arrays, no allocation, no
 * host synchronisation).  Any split is allowed: a chunk may continue from a
 * state whose pending block is partial, and zero-length updates are no-ops.
 * When the continued byte stream is 16-byte aligned in memory (data at
 * p with (p - num) 16-byte aligned: e.g. a chunk's mapped content appended
 * in place), every block after the first is read by the fast vector path;
 * otherwise blocks are gathered bytewise (correct, slower). */
int  cio_sha1_update_batch_dev(const void *dev_base, const uint64_t *dev_offs,
                               const uint64_t *dev_lens, cio_sha1_state *dev_states,
                               size_t n, void *stream);

/* SHA1_Final of every state into dev_digests + 20 i (big-endian).  The
 * states are NOT modified, so each stays the pre-Final context and can be
 * updated further (cio_sha1_hash's export, src/cio_sha1.c:41-57). */
int  cio_sha1_final_batch_dev(const cio_sha1_state *dev_states, uint8_t *dev_digests,
                              size_t n, void *stream);

/* ---- diagnostics -------------------------------------------------------- */

/* Read-only stream over floor(bytes / 4096) * 4096 bytes of dev_base with the
 * CRC kernel's grid and load pattern (no CRC): the practical HBM-read ceiling
 * the CRC kernel is measured against.  Asynchronous on `stream`. */
int  cio_gpu_read_stream(const void *dev_base, uint64_t bytes, void *stream);

/* The same on `workgroups` 1024-thread workgroups (0 = one per CU, <= 4096):
 * the ceiling for a plan that runs cio_crc32_plan_workgroups(plan) of them. */
int  cio_gpu_read_stream_grid(const void *dev_base, uint64_t bytes, uint32_t workgroups, void *stream);

/* ---- timing helpers (HIP events on a given stream) --------------------- */

void  *cio_gpu_event_create(void);
void   cio_gpu_event_destroy(void *ev);
int    cio_gpu_event_record(void *ev, void *stream);
float  cio_gpu_event_elapsed_ms(void *start, void *stop);   /* syncs stop */
int    cio_gpu_stream_sync(void *stream);

#ifdef __cplusplus
}
#endif

#endif /* CIO_CRC32_GPU_H */
