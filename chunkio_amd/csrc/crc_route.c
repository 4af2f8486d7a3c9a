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

const char *cioa_diag_getenv(const char *name)
{
    const char *gate = getenv("CIO_GPU_DIAG");
    if (!gate || strcmp(gate, "1") != 0) {
        return NULL;
    }
    return getenv(name);
}

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
 * Both engines at once.  With the split route on (default; CIOA_SPLIT_ROUTE=0
 * or cio_crc32_set_split_route(0) turn it off, and so does any explicit
 * threshold -- cio_crc32_set_cpu_max / CIOA_CPU_CRC_MAX: the caller chose an
 * engine) a large batch runs on the GPU and on the host at the same time: the
 * GPU part (the first chunks) on a helper thread, on the caller's device list
 * or its current device, and a suffix of whole chunks on the caller's
 * cio_crc32_host_threads() host threads, sized so both finish together:
 *
 *   B_host / r_host = F_gpu + (B - B_host) / (G r_gpu)
 *
 * The rates are learned: every split measures the host part's rate and the
 * GPU part's rate *while the other engine runs* (the GPU path's copy and
 * pread threads share the host's cores and memory with the CRC threads, so
 * the concurrent rates are not the solo ones), per host thread count and
 * source (memory / file), and the next split of that kind is sized with their
 * running average.  The first split of a kind starts from the model (memory
 * min(T x 36, 131) GB/s, files min(T x 22, 131) GB/s, GPU 54.7 GB/s per
 * device).  A split is taken when it gives the GPU at least kMinGpuShare
 * bytes and is predicted to finish before the better engine alone; this
 * covers batches the threshold sends to the GPU (one host thread: the caller
 * joins in) and batches it keeps on the host (T threads outrun one PCIe link,
 * and the GPU adds its share while the host is less than kMaxHostOverGpu
 * times faster).  Results are the same as either engine alone.  Measured on
 * the 1000 perf files (profiles/r05/split_probe_r05j*.txt). */
static const double kCpuThreadFdGBps = 22.0;
static const double kMinGpuShare = 32e6;
/* A host-routed batch is shared only while the host's (learned, concurrent)
 * rate is below this multiple of the GPUs': the GPU path's copy and pread
 * threads slow the host CRC threads, which pays while the GPU adds a large
 * share and not once the host is far faster.  Verify of the 1000 perf files
 * (profiles/r05/split_probe_r05j*.txt): host/GPU 0.35 (1 thread) +32%, 1.2
 * (4) +40%, 2.3 (8) +9-15%, 3.6-3.9 (16) -5-7%. */
static const double kMaxHostOverGpu = 3.0;
enum { kMaxT = 64 };
static double g_rh[2][kMaxT + 1];        /* learned host rate in a split, GB/s (0: none yet) */
static double g_rg[2];                   /* learned GPU rate per device in a split, GB/s */
static int g_rg_seen[2];                 /* GPU parts seen per kind; the first is not learned from */

int cio_crc32_split_route(void)
{
    const int v = __atomic_load_n(&g_split, __ATOMIC_ACQUIRE);
    if (v >= 0) {
        return v;
    }
    const char *r = getenv("CIOA_SPLIT_ROUTE");     /* "0" off, "2" forced (tests), else on */
    return r && strcmp(r, "0") == 0 ? 0 : r && strcmp(r, "2") == 0 ? 2 : 1;
}

void cio_crc32_set_split_route(int on)
{
    /* 0 off, 1 on, 2 forced: every batch of two or more chunks split, the
     * GPU taking at least its first chunk (tests) */
    __atomic_store_n(&g_split, on == 2 ? 2 : on ? 1 : 0, __ATOMIC_RELEASE);
}

static double ld_rate(const double *p)
{
    double v;
    __atomic_load(p, &v, __ATOMIC_RELAXED);
    return v;
}

/* Running average of a rate, clamped to [model / kLearnBand, model x
 * kLearnBand]: one outlier (a cold runtime, a host under other load) cannot
 * push the route so far off its model that it never splits again and so never
 * measures again. */
static const double kLearnBand = 4.0;

static void learn(double *p, double x, double model)
{
    const double lo = model / kLearnBand, hi = model * kLearnBand;
    x = x < lo ? lo : x > hi ? hi : x;
    const double old = ld_rate(p);
    double v = old > 0 ? 0.5 * old + 0.5 * x : x;
    __atomic_store(p, &v, __ATOMIC_RELAXED);
}

static void relax(double *p, double model)
{
    const double old = ld_rate(p);
    if (old > 0 && old < model) {
        double v = old + 0.1 * (model - old);
        __atomic_store(p, &v, __ATOMIC_RELAXED);
    }
}

/* Test hook (not in the public header): set the learned GPU rate of a kind
 * (0 memory, 1 files), GB/s per device; 0 forgets it. */
void cioa_debug_split_set_gpu_rate(int fd, double gbps)
{
    __atomic_store(&g_rg[fd ? 1 : 0], &gbps, __ATOMIC_RELAXED);
}

static double host_model(int t, int fd)
{
    const double m = t * (fd ? kCpuThreadFdGBps : kCpuThreadGBps);
    return m < kCpuMemGBps ? m : kCpuMemGBps;
}

static double host_rate(int t, int fd)
{
    const double l = ld_rate(&g_rh[fd][t]);
    return l > 0 ? l : host_model(t, fd);
}

static double gpu_rate(int fd)
{
    const double l = ld_rate(&g_rg[fd]);
    return l > 0 ? l : kGpuGBps;
}

void cio_crc32_split_rates(double *out, int n)
{
    /* {host mem T=1, host fd T=1, host mem T, host fd T, gpu mem, gpu fd} for
     * T = cio_crc32_host_threads(): what the next split would be sized with */
    const int t = cio_crc32_host_threads();
    const double v[6] = {host_rate(1, 0), host_rate(1, 1), host_rate(t, 0), host_rate(t, 1), gpu_rate(0), gpu_rate(1)};
    for (int i = 0; i < n && i < 6; i++) {
        out[i] = v[i];
    }
}

void cio_crc32_split_forget(void)
{
    double z = 0;
    for (int f = 0; f < 2; f++) {
        for (int t = 0; t <= kMaxT; t++) {
            __atomic_store(&g_rh[f][t], &z, __ATOMIC_RELAXED);
        }
        __atomic_store(&g_rg[f], &z, __ATOMIC_RELAXED);
        __atomic_store_n(&g_rg_seen[f], 0, __ATOMIC_RELAXED);
    }
}

/* Whether a GPU is visible (checked once; a host-routed batch is only shared
 * with one that exists). */
static int g_hip_probes;

void cioa_note_hip_probe(void)
{
    __atomic_fetch_add(&g_hip_probes, 1, __ATOMIC_RELAXED);
}

/* Test hook (not in the public header): how often the route and the sync
 * jobs asked the HIP runtime about devices.  A process whose batches all stay
 * on the host must never have asked. */
int cioa_debug_hip_probes(void)
{
    return __atomic_load_n(&g_hip_probes, __ATOMIC_RELAXED);
}

static int gpu_present(void)
{
    static int v = -1;
    int x = __atomic_load_n(&v, __ATOMIC_ACQUIRE);
    if (x < 0) {
        cioa_note_hip_probe();
        x = cio_gpu_device_count() > 0;
        __atomic_store_n(&v, x, __ATOMIC_RELEASE);
    }
    return x;
}

/* The GPU prefix of a split: chunks [0, k) on the GPU, [k, n) on the host;
 * k == n: the GPU alone, k == 0: the host alone. */
static size_t split_point(const size_t *lens, size_t n, int ndev_distinct, int fd, int gpu_bound)
{
    size_t explicit_max;
    const int mode = cio_crc32_split_route();
    const int have_max = explicit_cpu_max(&explicit_max);
    if (mode == 0 || n < 2 || (have_max && explicit_max == 0)) {
        return gpu_bound ? n : 0;      /* (an explicit threshold of 0: the GPU alone) */
    }
    if (mode != 2 && have_max && !(gpu_bound && __atomic_load_n(&g_split, __ATOMIC_ACQUIRE) == 1)) {
        /* an explicit threshold picks one engine, unless the caller also
         * turned the split on: then a batch the threshold sends to the GPU
         * may still be shared */
        return gpu_bound ? n : 0;
    }
    double total = 0;
    for (size_t i = 0; i < n; i++) {
        total += (double) lens[i];
    }
    if (mode != 2 && total < kMinGpuShare) {
        return gpu_bound ? n : 0;      /* no split could give the GPU its minimum share */
    }
    const int t = cio_crc32_host_threads();
    const double r_host = host_rate(t, fd) * 1e9;
    const double r_gpu = (ndev_distinct > 1 ? ndev_distinct : 1) * gpu_rate(fd) * 1e9;
    const double f = kGpuFixedUs * 1e-6;
    if (mode != 2 && !gpu_bound && r_host >= kMaxHostOverGpu * r_gpu) {
        /* The host alone (see kMaxHostOverGpu).  No split means no new GPU
         * sample, so a GPU rate learned too low would keep the route off for
         * good: each such decision moves the learned rate a tenth of the way
         * back to the model, and the route tries a split again once it has
         * recovered (the next split measures afresh). */
        relax(&g_rg[fd], kGpuGBps);
        return 0;
    }
    const double b_host = (f + total / r_gpu) / (1.0 / r_host + 1.0 / r_gpu);
    const double t_split = b_host / r_host;
    const double t_alone = gpu_bound ? f + total / r_gpu : total / r_host;
    if (mode != 2 && (total - b_host < kMinGpuShare || t_split >= t_alone)) {
        return gpu_bound ? n : 0;
    }
    /* Only now, with a split worth taking, ask whether a GPU exists: a batch
     * the size checks keep on the host never starts the HIP runtime. */
    if (!gpu_bound && !gpu_present()) {
        return 0;                      /* host-routed, and no GPU to share with */
    }
    size_t k = n;
    double acc = 0;
    while (k > 1 && acc + (double) lens[k - 1] <= b_host) {
        acc += (double) lens[--k];
    }
    return k;
}

/* Test hook (not in the public header; no device needed for a batch the
 * threshold sends to the GPU): the split point split_point() picks. */
size_t cioa_debug_split_point(const size_t *lens, size_t n, int ndev_distinct, int fd, int gpu_bound)
{
    return split_point(lens, n, ndev_distinct, fd, gpu_bound);
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
    double secs;
    char err[512];
    double timing[6];
};

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + (double) ts.tv_nsec * 1e-9;
}

static void *gpu_part_run(void *arg)
{
    struct gpu_part *g = (struct gpu_part *) arg;
    const double t0 = now_s();
    g->rc = g->fds ? cio_crc32_batch_fd_multi(g->fds, g->foffs, g->lens, g->seeds, g->out, g->n, g->devices, g->ndev)
                   : cio_crc32_batch_host_multi(g->bufs, g->lens, g->seeds, g->out, g->n, g->devices, g->ndev);
    g->secs = now_s() - t0;
    if (g->rc != CIO_OK) {
        snprintf(g->err, sizeof(g->err), "%s", cio_gpu_last_error());
    } else {
        (void) cio_gpu_pipe_last_timing(g->timing, 6);
    }
    return NULL;
}

/* Chunks [0, k) on the GPU (helper thread), [k, n) on the host (this thread).
 * host_routed: the threshold had put the whole batch on the host, so a GPU
 * part that fails is redone on the host instead of failing the batch. */
static int run_split(const void *const *bufs, const int *fds, const uint64_t *foffs, const size_t *lens,
                     const uint32_t *seeds, uint32_t *out_raw, size_t n, size_t k, const int *devices, int ndev,
                     int host_routed)
{
    int cur = -1;
    const int gdev = devices ? distinct_devices(devices, ndev) : 1;
    if (!devices || ndev <= 0) {
        /* the helper thread must use the caller's current device */
        cur = cio_gpu_get_device();
        if (cur < 0) {
            if (host_routed) {
                return fds ? cio_crc32_batch_fd_cpu(fds, foffs, lens, seeds, out_raw, n, cio_crc32_host_threads())
                           : cio_crc32_batch_cpu(bufs, lens, seeds, out_raw, n, cio_crc32_host_threads());
            }
            return cioa_fail_msg("cioa_crc_route", "no current HIP device");
        }
        devices = &cur;
        ndev = 1;
    }
    struct gpu_part g = {bufs, fds, foffs, lens, seeds, out_raw, k, devices, ndev, CIO_ERROR, 0, {0}, {0}};
    pthread_t th;
    if (pthread_create(&th, NULL, gpu_part_run, &g) != 0) {
        return cioa_fail_msg("cioa_crc_route", "pthread_create failed");
    }
    const int t = cio_crc32_host_threads();
    const double t0 = now_s();
    const int rc_host = fds ? cio_crc32_batch_fd_cpu(fds + k, foffs + k, lens + k, seeds ? seeds + k : NULL,
                                                     out_raw + k, n - k, t)
                            : cio_crc32_batch_cpu(bufs + k, lens + k, seeds ? seeds + k : NULL, out_raw + k, n - k, t);
    const double t_host = now_s() - t0;
    pthread_join(th, NULL);
    if (g.rc != CIO_OK) {
        if (host_routed && rc_host == CIO_OK) {
            /* redo the GPU's share where the threshold had put it */
            return fds ? cio_crc32_batch_fd_cpu(fds, foffs, lens, seeds, out_raw, k, t)
                       : cio_crc32_batch_cpu(bufs, lens, seeds, out_raw, k, t);
        }
        return cioa_fail_msg("cioa_crc_route: GPU part", g.err);
    }
    double hb = 0, gb = 0;
    for (size_t i = 0; i < n; i++) {
        *(i < k ? &gb : &hb) += (double) lens[i];
    }
    const int fd = fds != NULL;
    if (rc_host == CIO_OK && hb >= 8e6 && t_host > 0) {
        learn(&g_rh[fd][t], hb / t_host / 1e9, host_model(t, fd));
    }
    /* The first GPU part of a kind also pays the runtime's, the pipeline's and
     * the pinned buffers' set-up: it is not a rate sample. */
    const int first_gpu = __atomic_fetch_add(&g_rg_seen[fd], 1, __ATOMIC_RELAXED) == 0;
    const double tg = g.secs - kGpuFixedUs * 1e-6;
    if (!first_gpu && gb >= 8e6 && tg > 0.5 * g.secs) {
        learn(&g_rg[fd], gb / tg / 1e9 / gdev, kGpuGBps);
    }
    if (getenv("CIOA_ROUTE_DEBUG")) {
        fprintf(stderr, "split route: %zu chunks, gpu %zu (%.1f MB), host %zu (%.1f MB, %d threads): "
                        "host %.2f ms, gpu %.2f ms; next: host %.1f GB/s, gpu %.1f GB/s\n", n, k, gb / 1e6, n - k,
                hb / 1e6, t, t_host * 1e3, g.secs * 1e3, host_rate(t, fd), gpu_rate(fd));
    }
    cioa_pipe_timing_set(g.timing);
    return rc_host;
}

void cioa_crc_route_plan(const size_t *lens, size_t n, const int *devices, int ndev, int fd, cioa_route_plan *plan)
{
    plan->gpu_bound = n > 0 && !route_to_cpu(lens, n, devices, ndev);
    plan->k = n > 0 ? split_point(lens, n, devices ? distinct_devices(devices, ndev) : 1, fd, plan->gpu_bound) : 0;
}

int cioa_crc_batch_route_planned(const void *const *bufs, const size_t *lens, const uint32_t *seeds,
                                 uint32_t *out_raw, size_t n, const int *devices, int ndev,
                                 const cioa_route_plan *plan)
{
    if (n == 0) {
        return CIO_OK;
    }
    const size_t k = plan->k;
    if (k == 0) {
        return cio_crc32_batch_cpu(bufs, lens, seeds, out_raw, n, cio_crc32_host_threads());
    }
    if (k < n) {
        return run_split(bufs, NULL, NULL, lens, seeds, out_raw, n, k, devices, ndev, !plan->gpu_bound);
    }
    return cio_crc32_batch_host_multi(bufs, lens, seeds, out_raw, n, devices, ndev);
}

int cioa_crc_batch_route(const void *const *bufs, const size_t *lens, const uint32_t *seeds, uint32_t *out_raw,
                         size_t n, const int *devices, int ndev)
{
    cioa_route_plan plan;
    cioa_crc_route_plan(lens, n, devices, ndev, 0, &plan);
    return cioa_crc_batch_route_planned(bufs, lens, seeds, out_raw, n, devices, ndev, &plan);
}

int cioa_crc_fd_route(const int *fds, const uint64_t *foffs, const size_t *lens, const uint32_t *seeds,
                      uint32_t *out_raw, size_t n, const int *devices, int ndev)
{
    if (n == 0) {
        return CIO_OK;
    }
    const int gpu_bound = !route_to_cpu(lens, n, devices, ndev);
    const size_t k = split_point(lens, n, devices ? distinct_devices(devices, ndev) : 1, 1, gpu_bound);
    if (k == 0) {
        return cio_crc32_batch_fd_cpu(fds, foffs, lens, seeds, out_raw, n, cio_crc32_host_threads());
    }
    if (k < n) {
        return run_split(NULL, fds, foffs, lens, seeds, out_raw, n, k, devices, ndev, !gpu_bound);
    }
    return cio_crc32_batch_fd_multi(fds, foffs, lens, seeds, out_raw, n, devices, ndev);
}
