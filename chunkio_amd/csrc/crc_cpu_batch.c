/*
 * crc_cpu_batch.c -- the host CRC batch: crc_update (crc32_host.c, the
 * drop-in for deps/crc32/crc32.c:337-390) over many independent chunks, on
 * up to `threads` host threads.
 *
 * The reference computes one chunk's CRC on the calling thread
 * (src/cio_file.c:66-94 for a whole region, :97-113 per write).  This is the
 * same arithmetic spread over a thread pool so that a batch of host-resident
 * chunks -- a verify-on-load scan, a batched sync -- can be CRC'd on the CPU
 * when that is faster than shipping the bytes over PCIe to the GPU
 * (crc_route.c decides).  Chunks are cut into pieces of at most kPiece
 * bytes; pieces of consecutive small chunks are grouped into tasks of about
 * kTask bytes; threads claim tasks from one atomic counter; a chunk's
 * pieces are folded in order with cio_crc32_combine (x^(8 len) mod P), so a
 * single large chunk uses every thread and the result is bit-identical to
 * one crc_update over the whole chunk.
 *
 * File sources (fd, offset) are pread() through a per-thread buffer.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <crc32/crc32.h>
#include "chunkio_amd/cio_crc32_gpu.h"
#include "crc32_host.h"

enum {
    kPiece = 1 << 20,           /* max bytes of one piece (a chunk splits above it) */
    kTask = 256 << 10,          /* min bytes of one claimed task (small chunks grouped) */
    kReadBuf = 256 << 10,       /* pread buffer per thread for file sources */
    kMaxThreads = 64,
};

struct piece {
    uint64_t off;               /* within the chunk */
    uint64_t len;
    uint32_t chunk;
};

struct cpu_job {
    const void *const *bufs;    /* memory sources, or NULL */
    const int *fds;             /* file sources, or NULL */
    const uint64_t *foffs;
    const uint32_t *seeds;
    const struct piece *pieces;
    const size_t *task_lo;      /* task t = pieces [task_lo[t], task_lo[t + 1]) */
    size_t ntasks;
    uint32_t *praw;             /* raw state per piece */
    size_t next;                /* atomic: next task to claim */
    int failed;                 /* atomic: a file range could not be read */
};

/* pread bounce buffer per thread (file sources), freed when its thread
 * exits (a caller thread routes fd batches here too, and services spawn and
 * end such threads). */
static pthread_key_t g_rb_key;
static pthread_once_t g_rb_once = PTHREAD_ONCE_INIT;

static void rb_key_make(void)
{
    (void) pthread_key_create(&g_rb_key, free);
}

static unsigned char *thread_readbuf(void)
{
    (void) pthread_once(&g_rb_once, rb_key_make);
    unsigned char *b = pthread_getspecific(g_rb_key);
    if (!b && (b = malloc(kReadBuf)) != NULL && pthread_setspecific(g_rb_key, b) != 0) {
        free(b);
        b = NULL;
    }
    return b;
}

static int run_piece(const struct cpu_job *j, const struct piece *pc, uint32_t *out)
{
    /* the chunk's first piece starts from its seed, later ones from 0 (folded in) */
    const crc_t seed = pc->off == 0 ? (crc_t) (j->seeds ? j->seeds[pc->chunk] : 0xffffffffu) : 0;
    if (!j->fds) {
        const unsigned char *p = (const unsigned char *) j->bufs[pc->chunk] + pc->off;
        *out = (uint32_t) crc_update(seed, p, (size_t) pc->len);
        return 0;
    }
    unsigned char *t_readbuf = thread_readbuf();
    if (!t_readbuf) {
        return -1;
    }
    crc_t c = seed;
    uint64_t done = 0;
    while (done < pc->len) {
        const size_t want = pc->len - done < kReadBuf ? (size_t) (pc->len - done) : kReadBuf;
        const ssize_t r = pread(j->fds[pc->chunk], t_readbuf, want, (off_t) (j->foffs[pc->chunk] + pc->off + done));
        if (r < 0 && errno == EINTR) {
            continue;
        }
        if (r <= 0) {
            return -1;
        }
        c = crc_update(c, t_readbuf, (size_t) r);
        done += (uint64_t) r;
    }
    *out = (uint32_t) c;
    return 0;
}

static void run_tasks(struct cpu_job *j)
{
    for (;;) {
        const size_t t = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        if (t >= j->ntasks) {
            return;
        }
        for (size_t k = j->task_lo[t]; k < j->task_lo[t + 1]; k++) {
            if (run_piece(j, &j->pieces[k], &j->praw[k]) != 0) {
                __atomic_store_n(&j->failed, 1, __ATOMIC_RELAXED);
            }
        }
    }
}

/* ---- persistent worker pool (started on first use, grown on demand) ------ */

static pthread_mutex_t g_job_mu = PTHREAD_MUTEX_INITIALIZER;    /* one batch at a time */
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t g_cv = PTHREAD_COND_INITIALIZER;
static pthread_cond_t g_done_cv = PTHREAD_COND_INITIALIZER;
static int g_started;                 /* workers running */
static uint64_t g_gen;                /* batch generation */
static struct cpu_job *g_job;
static int g_want;                    /* workers taking part in this batch */
static int g_pending;
static int g_stop;                    /* library unload / process exit: workers leave */
static pthread_t g_tid[kMaxThreads];  /* joinable, so unload can wait for them */

struct worker_arg {
    int idx;
    uint64_t seen;              /* the generation current when it was created */
};

static void *worker(void *arg)
{
    const struct worker_arg wa = *(const struct worker_arg *) arg;
    free(arg);
    const int idx = wa.idx;
    uint64_t seen = wa.seen;    /* so a worker started for this batch joins it */
    pthread_mutex_lock(&g_mu);
    for (;;) {
        while (g_gen == seen && !g_stop) {
            pthread_cond_wait(&g_cv, &g_mu);
        }
        if (g_gen == seen) {
            /* stopping, and no batch published since this worker's last one */
            pthread_mutex_unlock(&g_mu);
            return NULL;
        }
        /* A published batch is served even when the stop came with it:
         * pool_run counted this worker in g_pending and waits for it. */
        seen = g_gen;
        if (idx >= g_want) {
            continue;
        }
        struct cpu_job *j = g_job;
        pthread_mutex_unlock(&g_mu);
        run_tasks(j);
        pthread_mutex_lock(&g_mu);
        if (--g_pending == 0) {
            pthread_cond_signal(&g_done_cv);
        }
    }
    return NULL;
}

/* The pool's detached workers run this library's code: on dlclose (or at
 * exit) they are told to leave and waited for, at most 2 s, so none is left
 * executing unmapped code.  A worker in the middle of a batch finishes its
 * tasks first. */
__attribute__((destructor)) static void pool_stop(void)
{
    pthread_mutex_lock(&g_mu);
    g_stop = 1;
    const int n = g_started;
    pthread_cond_broadcast(&g_cv);
    pthread_mutex_unlock(&g_mu);
    struct timespec dl;
    clock_gettime(CLOCK_REALTIME, &dl);
    dl.tv_sec += 2;
    for (int i = 0; i < n; i++) {
        /* joined, not counted: a worker is only gone once it has returned.
         * One worker past the deadline does not stop the others from being
         * joined (after it, each join only collects a worker already gone). */
        (void) pthread_timedjoin_np(g_tid[i], NULL, &dl);
    }
}

/* Runs j on the caller plus up to helpers pool workers; returns after all
 * of them are done with it. */
static void pool_run(struct cpu_job *j, int helpers)
{
    pthread_mutex_lock(&g_mu);
    if (g_stop) {
        helpers = 0;          /* (a batch during unload: the caller alone) */
    }
    while (g_started < helpers) {
        pthread_t th;
        pthread_attr_t at;
        struct worker_arg *wa = malloc(sizeof(*wa));
        if (!wa) {
            break;
        }
        wa->idx = g_started;
        wa->seen = g_gen;
        pthread_attr_init(&at);
        const int ok = g_started < kMaxThreads && pthread_create(&th, &at, worker, wa) == 0;
        pthread_attr_destroy(&at);
        if (!ok) {
            free(wa);
            break;
        }
        g_tid[g_started++] = th;
    }
    if (helpers > g_started) {
        helpers = g_started;
    }
    g_job = j;
    g_want = helpers;
    g_pending = helpers;
    g_gen++;
    pthread_cond_broadcast(&g_cv);
    pthread_mutex_unlock(&g_mu);
    run_tasks(j);
    pthread_mutex_lock(&g_mu);
    while (g_pending > 0) {
        pthread_cond_wait(&g_done_cv, &g_mu);
    }
    g_job = NULL;
    pthread_mutex_unlock(&g_mu);
}

static int cpu_batch(const void *const *bufs, const int *fds, const uint64_t *foffs, const size_t *lens,
                     const uint32_t *seeds, uint32_t *out_raw, size_t n, int threads, const char *what)
{
    if (n == 0) {
        return CIO_OK;
    }
    if (threads < 1) {
        threads = 1;
    }
    if (threads > kMaxThreads) {
        threads = kMaxThreads;
    }
    size_t np = 0;
    uint64_t total = 0;
    for (size_t i = 0; i < n; i++) {
        np += lens[i] ? (lens[i] + kPiece - 1) / kPiece : 1;
        total += lens[i];
    }
    const uint64_t tasks_wanted = total / kTask + 1;
    /* one thread, or a batch too small to share: the calling thread alone,
     * chunk by chunk, exactly the reference's loop */
    if (threads == 1 || tasks_wanted < 2) {
        struct cpu_job j = {bufs, fds, foffs, seeds, NULL, NULL, 0, NULL, 0, 0};
        for (size_t i = 0; i < n; i++) {
            const struct piece pc = {0, lens[i], (uint32_t) i};
            if (run_piece(&j, &pc, &out_raw[i]) != 0) {
                return cioa_fail_msg(what, "short read from a file source");
            }
        }
        return CIO_OK;
    }
    struct piece *pieces = malloc(np * sizeof(*pieces));
    size_t *task_lo = malloc((np + 1) * sizeof(*task_lo));
    uint32_t *praw = malloc(np * sizeof(*praw));
    if (!pieces || !task_lo || !praw) {
        free(pieces);
        free(task_lo);
        free(praw);
        return cioa_fail_msg(what, "out of memory");
    }
    size_t k = 0, nt = 0;
    uint64_t acc = 0;
    for (size_t i = 0; i < n; i++) {
        uint64_t off = 0;
        do {
            const uint64_t len = lens[i] - off < (uint64_t) kPiece ? lens[i] - off : (uint64_t) kPiece;
            if (acc == 0) {
                task_lo[nt++] = k;
            }
            pieces[k++] = (struct piece) {off, len, (uint32_t) i};
            acc += len + 64;                 /* + a per-piece cost, so empty chunks group too */
            if (acc >= kTask) {
                acc = 0;
            }
            off += len;
        } while (off < lens[i]);
    }
    task_lo[nt] = k;
    struct cpu_job j = {bufs, fds, foffs, seeds, pieces, task_lo, nt, praw, 0, 0};
    int helpers = threads - 1;
    if ((size_t) helpers > nt - 1) {
        helpers = (int) (nt - 1);
    }
    pthread_mutex_lock(&g_job_mu);
    pool_run(&j, helpers);
    pthread_mutex_unlock(&g_job_mu);
    int rc = CIO_OK;
    if (j.failed) {
        rc = cioa_fail_msg(what, "short read from a file source");
    } else {
        for (size_t p = 0; p < np; p++) {
            const struct piece *pc = &pieces[p];
            out_raw[pc->chunk] = pc->off == 0 ? praw[p] : cio_crc32_combine(out_raw[pc->chunk], praw[p], pc->len);
        }
    }
    free(pieces);
    free(task_lo);
    free(praw);
    return rc;
}

int cio_crc32_batch_cpu(const void *const *bufs, const size_t *lens, const uint32_t *seeds, uint32_t *out_raw,
                        size_t n, int threads)
{
    if (n && (!bufs || !lens || !out_raw)) {
        return cioa_fail_msg("cio_crc32_batch_cpu", "null argument");
    }
    if (n >= 0xffffffffull) {
        return cioa_fail_msg("cio_crc32_batch_cpu", "too many chunks");
    }
    return cpu_batch(bufs, NULL, NULL, lens, seeds, out_raw, n, threads, "cio_crc32_batch_cpu");
}

int cio_crc32_batch_fd_cpu(const int *fds, const uint64_t *foffs, const size_t *lens, const uint32_t *seeds,
                           uint32_t *out_raw, size_t n, int threads)
{
    if (n && (!fds || !foffs || !lens || !out_raw)) {
        return cioa_fail_msg("cio_crc32_batch_fd_cpu", "null argument");
    }
    if (n >= 0xffffffffull) {
        return cioa_fail_msg("cio_crc32_batch_fd_cpu", "too many chunks");
    }
    return cpu_batch(NULL, fds, foffs, lens, seeds, out_raw, n, threads, "cio_crc32_batch_fd_cpu");
}
