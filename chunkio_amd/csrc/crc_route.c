/*
 * crc_route.c -- where the chunk layer's host-memory CRCs run.
 *
 * The chunk layer's verify/sync batches (cio_verify.c, cio_sync.c,
 * cioa_chunk.c) hold chunk bytes in host memory (mmap'd files,
 * src/cio_file_unix.c:100) or in files.  Two engines can CRC them, with
 * identical results (both compute crc_update(seed, bytes)):
 *
 *   - the GPU host batch (cio_crc32_batch_host_multi / _fd_multi): a fixed
 *     cost per call (plan image + bytes over PCIe, launches, the states back,
 *     two synchronisations), then the PCIe rate per device;
 *   - the host batch (cio_crc32_batch_cpu / _fd_cpu, crc_cpu_batch.c): the
 *     library's crc_update (VPCLMULQDQ folding) on cio_crc32_host_threads()
 *     threads, no fixed cost to speak of, a per-thread rate from DRAM up to
 *     the socket's memory bandwidth.
 *
 * cioa_crc_batch_route() sends a batch whose total size is at most
 * cio_crc32_cpu_max() bytes to the host, everything larger to the GPU.  The
 * default threshold comes from that cost model with rates measured on the
 * MI355X box (bench.py's `host_route` leg, profiles/r04/):
 *
 *   GPU:  kGpuFixedUs + B / (G x kGpuGBps)      G = distinct devices in the call
 *   host: B / min(T x kCpuThreadGBps, kCpuMemGBps)
 *
 * so the host wins below B* = kGpuFixedUs / (1/r_host - 1/r_gpu), and for
 * every size once r_host >= r_gpu.  With chunkio's one thread (T = 1, the
 * default: the reference is single-threaded and so is Fluent Bit's caller)
 * B* is ~17 MB per device (measured crossovers: between 52 and 105 MB on
 * the fast box, between 13 and 26 MB on the slow one).  With T >= 2 host threads the host's DRAM rate
 * already beats one PCIe link, so host-resident batches stay on the CPU: the
 * GPU path pays off for host-resident chunks only when the caller cannot
 * spare cores.  CIOA_CPU_CRC_MAX / cio_crc32_set_cpu_max() override the
 * threshold (0 = always the GPU); CIOA_HOST_CRC_THREADS /
 * cio_crc32_set_host_threads() set T.  The public cio_crc32_batch_* entry
 * points never route.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <crc32/crc32.h>
#include "chunkio_amd/cio_crc32_gpu.h"
#include "crc32_host.h"

/* Cost-model rates (see the header comment), measured on MI355X boxes by
 * tools/route_batch.py (batches of 1..1024 x 400 KB in DRAM-resident
 * pageable memory): the GPU host batch's least-squares fixed cost and rate
 * (profiles/r04/route_batch_r04d.json: 163.5 us, 54.7 GB/s), and
 * crc_update's rate on one thread and on 16, which differ by box (r04a:
 * 47.6 / 396 GB/s; r04d: 27.4 / 131 GB/s over the whole sweep).  The
 * one-thread rate is the slower box's where the crossover lies -- 13 to
 * 52 MB batches run at 36-40 GB/s there (its 27.4 GB/s fit is pulled down
 * by the 100-400 MB batches) -- so the model's crossover, ~17 MB, falls
 * between that box's measured 13 MB (host faster) and 26 MB (GPU faster)
 * and below the faster box's 52-105 MB: an ambiguous batch still goes to
 * the GPU and leaves the host's cores to the caller. */
static const double kGpuFixedUs = 163.5;
static const double kGpuGBps = 54.7;
static const double kCpuThreadGBps = 36.0;
static const double kCpuMemGBps = 131.0;

static size_t g_cpu_max;
static int g_cpu_max_set;
static int g_split = -1;          /* split route: -1 not set (environment), 0 / 1 */
static int g_threads;
static int g_threads_set;

int cio_crc32_host_threads(void)
{
    if (__atomic_load_n(&g_threads_set, __ATOMIC_ACQUIRE)) {
        return __atomic_load_n(&g_threads, __ATOMIC_RELAXED);
    }
    const char *r = getenv("CIOA_HOST_CRC_THREADS");
    if (r && *r) {
        const int v = atoi(r);
        if (v >= 1 && v <= 64) {
            return v;
        }
    }
    return 1;
}

void cio_crc32_set_host_threads(int threads)
{
    if (threads < 1) {
        threads = 1;
    }
    if (threads > 64) {
        threads = 64;
    }
    __atomic_store_n(&g_threads, threads, __ATOMIC_RELAXED);
    __atomic_store_n(&g_threads_set, 1, __ATOMIC_RELEASE);
}

/* The model's crossover for T host threads against G devices. */
static size_t model_cpu_max(int threads, int ndev)
{
    double r_host = threads * kCpuThreadGBps;
    if (r_host > kCpuMemGBps) {
        r_host = kCpuMemGBps;
    }
    const double r_gpu = (ndev > 1 ? ndev : 1) * kGpuGBps;
    if (r_host >= r_gpu) {
        return SIZE_MAX;
    }
    const double b = kGpuFixedUs * 1e-6 / (1.0 / (r_host * 1e9) - 1.0 / (r_gpu * 1e9));
    return (size_t) b;
}

static int explicit_cpu_max(size_t *out)
{
    if (__atomic_load_n(&g_cpu_max_set, __ATOMIC_ACQUIRE)) {
        *out = __atomic_load_n(&g_cpu_max, __ATOMIC_RELAXED);
        return 1;
    }
    const char *r = getenv("CIOA_CPU_CRC_MAX");
    if (r && *r) {
        char *end = NULL;
        const unsigned long long v = strtoull(r, &end, 10);
        if (end && *end == '\0') {
            *out = (size_t) v;
            return 1;
        }
    }
    return 0;
}

size_t cio_crc32_cpu_max(void)
{
    size_t v;
    if (explicit_cpu_max(&v)) {
        return v;
    }
    return model_cpu_max(cio_crc32_host_threads(), 1);
}

void cio_crc32_set_cpu_max(size_t bytes)
{
    __atomic_store_n(&g_cpu_max, bytes, __ATOMIC_RELAXED);
    __atomic_store_n(&g_cpu_max_set, 1, __ATOMIC_RELEASE);
}

void cio_crc32_route_reset(void)
{
    __atomic_store_n(&g_cpu_max_set, 0, __ATOMIC_RELEASE);
    __atomic_store_n(&g_threads_set, 0, __ATOMIC_RELEASE);
    __atomic_store_n(&g_split, -1, __ATOMIC_RELEASE);
}

/* Distinct device ordinals in a *_multi device list (1 for the current device). */
static int distinct_devices(const int *devices, int ndev)
{
    int k = 0;
    for (int a = 0; a < ndev; a++) {
        int seen = 0;
        for (int b = 0; b < a && !seen; b++) {
            seen = devices[b] == devices[a];
        }
        k += !seen;
    }
    return k > 0 ? k : 1;
}

static int route_to_cpu(const size_t *lens, size_t n, const int *devices, int ndev)
{
    size_t max;
    if (!explicit_cpu_max(&max)) {
        max = model_cpu_max(cio_crc32_host_threads(), devices ? distinct_devices(devices, ndev) : 1);
    }
    size_t total = 0;
    for (size_t i = 0; i < n; i++) {
        total += lens[i];
        if (total > max) {
            return 0;
        }
    }
    return 1;
}

/* ---- split route --------------------------------------------------------
 *
 * A batch that goes to the GPU leaves the calling thread (and its
 * cio_crc32_host_threads() host CRC threads) waiting on the pipeline.  With
 * the split route on (default; CIOA_SPLIT_ROUTE=0 or cio_crc32_set_split_route
 * (0) turn it off, and so does an explicit cio_crc32_set_cpu_max(0): "all on
 * the GPU") the host takes a suffix of the batch at the same time: the
 * GPU part runs on a helper thread (on the caller's device list, or its
 * current device) while the caller CRCs its share with the host batch, sized
 * so both finish together under the cost model:
 *
 *   B_host / r_host = F_gpu + (B - B_host) / (G r_gpu)
 *
 * with r_host the host rate of this source (memory: min(T x 36, 131) GB/s;
 * files: min(T x 22, 131) GB/s, the pread path measured in bench.py's verify
 * leg).  Whole chunks only: the suffix is the last chunks whose total stays
 * within B_host.  Results are the same as either engine alone. */
static const double kCpuThreadFdGBps = 22.0;

int cio_crc32_split_route(void)
{
    const int v = __atomic_load_n(&g_split, __ATOMIC_ACQUIRE);
    if (v >= 0) {
        return v;
    }
    const char *r = getenv("CIOA_SPLIT_ROUTE");
    return !(r && strcmp(r, "0") == 0);
}

void cio_crc32_set_split_route(int on)
{
    __atomic_store_n(&g_split, on ? 1 : 0, __ATOMIC_RELEASE);
}

/* Diagnostic (CIOA_SPLIT_HOSTFAST=1, tools/split_probe.py): also split a
 * batch the model sends to the host because T host threads outrun the GPU,
 * giving the GPU the share the same equal-finish sizing assigns it. */
static int split_hostfast(void)
{
    const char *r = getenv("CIOA_SPLIT_HOSTFAST");     /* (read per batch: a probe toggles it) */
    return r && strcmp(r, "1") == 0;
}

/* First chunk of the host's suffix (n = no split). */
static size_t split_point(const size_t *lens, size_t n, int ndev_distinct, int fd)
{
    size_t explicit_max;
    if (!cio_crc32_split_route() || n < 2 || (explicit_cpu_max(&explicit_max) && explicit_max == 0)) {
        return n;    /* (an explicit threshold of 0 means every byte on the GPU) */
    }
    const int t = cio_crc32_host_threads();
    double r_host = t * (fd ? kCpuThreadFdGBps : kCpuThreadGBps);
    if (r_host > kCpuMemGBps) {
        r_host = kCpuMemGBps;
    }
    const double r_gpu = (ndev_distinct > 1 ? ndev_distinct : 1) * kGpuGBps;
    double total = 0;
    for (size_t i = 0; i < n; i++) {
        total += (double) lens[i];
    }
    const double b_host = (kGpuFixedUs * 1e-6 + total / (r_gpu * 1e9)) / (1.0 / (r_host * 1e9) + 1.0 / (r_gpu * 1e9));
    size_t k = n;
    double acc = 0;
    while (k > 1 && acc + (double) lens[k - 1] <= b_host) {
        acc += (double) lens[--k];
    }
    if (split_hostfast() && k == 1 && b_host >= total) {
        return 0;      /* (diagnostic path) the model gives the GPU nothing */
    }
    return k;
}

struct gpu_part {
    const void *const *bufs;
    const int *fds;
    const uint64_t *foffs;
    const size_t *lens;
    const uint32_t *seeds;
    uint32_t *out;
    size_t n;
    const int *devices;
    int ndev;
    int rc;
    char err[512];
    double timing[6];
};

static void *gpu_part_run(void *arg)
{
    struct gpu_part *g = (struct gpu_part *) arg;
    g->rc = g->fds ? cio_crc32_batch_fd_multi(g->fds, g->foffs, g->lens, g->seeds, g->out, g->n, g->devices, g->ndev)
                   : cio_crc32_batch_host_multi(g->bufs, g->lens, g->seeds, g->out, g->n, g->devices, g->ndev);
    if (g->rc != CIO_OK) {
        snprintf(g->err, sizeof(g->err), "%s", cio_gpu_last_error());
    } else {
        (void) cio_gpu_pipe_last_timing(g->timing, 6);
    }
    return NULL;
}

/* Chunks [0, k) on the GPU (helper thread), [k, n) on the host (this thread). */
static int run_split(const void *const *bufs, const int *fds, const uint64_t *foffs, const size_t *lens,
                     const uint32_t *seeds, uint32_t *out_raw, size_t n, size_t k, const int *devices, int ndev)
{
    int cur = -1;
    if (!devices || ndev <= 0) {
        /* the helper thread must use the caller's current device */
        cur = cio_gpu_get_device();
        if (cur < 0) {
            return cioa_fail_msg("cioa_crc_route", "no current HIP device");
        }
        devices = &cur;
        ndev = 1;
    }
    struct gpu_part g = {bufs, fds, foffs, lens, seeds, out_raw, k, devices, ndev, CIO_ERROR, {0}, {0}};
    pthread_t th;
    if (pthread_create(&th, NULL, gpu_part_run, &g) != 0) {
        return cioa_fail_msg("cioa_crc_route", "pthread_create failed");
    }
    const int t = cio_crc32_host_threads();
    struct timespec t0, t1, t2;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    const int rc_host = fds ? cio_crc32_batch_fd_cpu(fds + k, foffs + k, lens + k, seeds ? seeds + k : NULL,
                                                     out_raw + k, n - k, t)
                            : cio_crc32_batch_cpu(bufs + k, lens + k, seeds ? seeds + k : NULL, out_raw + k, n - k, t);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    pthread_join(th, NULL);
    clock_gettime(CLOCK_MONOTONIC, &t2);
    if (getenv("CIOA_ROUTE_DEBUG")) {
        double hb = 0, gb = 0;
        for (size_t i = 0; i < n; i++) {
            *(i < k ? &gb : &hb) += (double) lens[i];
        }
        fprintf(stderr, "split route: %zu chunks, gpu %zu (%.1f MB), host %zu (%.1f MB, %d threads): "
                        "host done %.2f ms, gpu done %.2f ms\n", n, k, gb / 1e6, n - k, hb / 1e6, t,
                (t1.tv_sec - t0.tv_sec) * 1e3 + (t1.tv_nsec - t0.tv_nsec) / 1e6,
                (t2.tv_sec - t0.tv_sec) * 1e3 + (t2.tv_nsec - t0.tv_nsec) / 1e6);
    }
    if (g.rc != CIO_OK) {
        return cioa_fail_msg("cioa_crc_route: GPU part", g.err);
    }
    cioa_pipe_timing_set(g.timing);
    return rc_host;
}

static int route_to_cpu_split(const size_t *lens, size_t n, const int *devices, int ndev)
{
    size_t m;
    if (split_hostfast() && !explicit_cpu_max(&m) && cio_crc32_host_threads() > 1) {
        return 0;
    }
    return route_to_cpu(lens, n, devices, ndev);
}

int cioa_crc_batch_route(const void *const *bufs, const size_t *lens, const uint32_t *seeds, uint32_t *out_raw,
                         size_t n, const int *devices, int ndev)
{
    if (n == 0) {
        return CIO_OK;
    }
    if (!route_to_cpu_split(lens, n, devices, ndev)) {
        const size_t k = split_point(lens, n, devices ? distinct_devices(devices, ndev) : 1, 0);
        if (k == 0) {
            return cio_crc32_batch_cpu(bufs, lens, seeds, out_raw, n, cio_crc32_host_threads());
        }
        if (k < n) {
            return run_split(bufs, NULL, NULL, lens, seeds, out_raw, n, k, devices, ndev);
        }
        return cio_crc32_batch_host_multi(bufs, lens, seeds, out_raw, n, devices, ndev);
    }
    return cio_crc32_batch_cpu(bufs, lens, seeds, out_raw, n, cio_crc32_host_threads());
}

int cioa_crc_fd_route(const int *fds, const uint64_t *foffs, const size_t *lens, const uint32_t *seeds,
                      uint32_t *out_raw, size_t n, const int *devices, int ndev)
{
    if (n == 0) {
        return CIO_OK;
    }
    if (!route_to_cpu_split(lens, n, devices, ndev)) {
        const size_t k = split_point(lens, n, devices ? distinct_devices(devices, ndev) : 1, 1);
        if (k == 0) {
            return cio_crc32_batch_fd_cpu(fds, foffs, lens, seeds, out_raw, n, cio_crc32_host_threads());
        }
        if (k < n) {
            return run_split(NULL, fds, foffs, lens, seeds, out_raw, n, k, devices, ndev);
        }
        return cio_crc32_batch_fd_multi(fds, foffs, lens, seeds, out_raw, n, devices, ndev);
    }
    return cio_crc32_batch_fd_cpu(fds, foffs, lens, seeds, out_raw, n, cio_crc32_host_threads());
}
