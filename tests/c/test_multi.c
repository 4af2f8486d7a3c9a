/*
 * The in-process multi-device host batches from C:
 * cio_crc32_batch_host_multi, cio_crc32_batch_fd_multi and
 * cio_crc32_split_host_multi over 1..4 device entries (all device 0 on a
 * one-GPU box: each entry still gets its own host thread, pipeline and
 * stream), plus several caller threads sharing the per-device pipeline pool.
 * Every result is compared with a bit-serial CRC-32 written here (reflected
 * 0xEDB88320, raw state in and out, as deps/crc32/crc32.c:337-390 computes),
 * so the check does not rest on the library's own crc_update.
 *
 * Needs a GPU; run by tests/test_c_api.py (-m gpu) and under the sanitizers
 * by tools/asan_check.sh.  Usage: test_multi <scratch dir>
 */
#include <fcntl.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <chunkio_amd/cio_crc32_gpu.h>

static int checks, failures;

#define CHECK(cond, ...)                                                 \
    do {                                                                 \
        checks++;                                                        \
        if (!(cond)) {                                                   \
            failures++;                                                  \
            fprintf(stderr, "FAILED %s:%d: ", __FILE__, __LINE__);       \
            fprintf(stderr, __VA_ARGS__);                                \
            fprintf(stderr, "\n");                                       \
        }                                                                \
    } while (0)

/* bit-serial CRC-32/IEEE on the raw (pre-inverted) state */
static uint32_t crc_bits(uint32_t crc, const uint8_t *p, size_t n)
{
    for (size_t i = 0; i < n; i++) {
        crc ^= p[i];
        for (int k = 0; k < 8; k++) {
            crc = (crc >> 1) ^ (0xEDB88320u & (0u - (crc & 1u)));
        }
    }
    return crc;
}

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;

static uint64_t rng(void)
{
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct batch {
    size_t n;
    uint8_t **bufs;
    size_t *lens;
    uint32_t *seeds;
    uint32_t *want;
};

/* n chunks: empty, 1..4096 B, up to 3 MiB, and one past a 64 MiB staging slot */
static void make_batch(struct batch *b, size_t n, int big)
{
    b->n = n;
    b->bufs = calloc(n, sizeof(*b->bufs));
    b->lens = calloc(n, sizeof(*b->lens));
    b->seeds = calloc(n, sizeof(*b->seeds));
    b->want = calloc(n, sizeof(*b->want));
    for (size_t i = 0; i < n; i++) {
        size_t len;
        switch (i % 5) {
        case 0: len = 0; break;
        case 1: len = 1 + rng() % 4096; break;
        case 2: len = 409600; break;
        default: len = rng() % (3u << 20); break;
        }
        if (big && i == n / 2) {
            len = (64u << 20) + 12345;
        }
        b->lens[i] = len;
        b->bufs[i] = malloc(len ? len : 1);
        for (size_t k = 0; k < len; k++) {
            b->bufs[i][k] = (uint8_t) rng();
        }
        b->seeds[i] = (i % 3) ? (uint32_t) rng() : 0xFFFFFFFFu;
        b->want[i] = crc_bits(b->seeds[i], b->bufs[i], len);
    }
}

static void free_batch(struct batch *b)
{
    for (size_t i = 0; i < b->n; i++) {
        free(b->bufs[i]);
    }
    free(b->bufs);
    free(b->lens);
    free(b->seeds);
    free(b->want);
}

static int same(const uint32_t *a, const uint32_t *b, size_t n)
{
    for (size_t i = 0; i < n; i++) {
        if (a[i] != b[i]) {
            fprintf(stderr, "  chunk %zu: 0x%08x != 0x%08x\n", i, a[i], b[i]);
            return 0;
        }
    }
    return 1;
}

static const int devs[4] = {0, 0, 0, 0};

static void test_host_multi(const struct batch *b)
{
    uint32_t *out = calloc(b->n, sizeof(uint32_t));
    for (int ndev = 1; ndev <= 4; ndev++) {
        memset(out, 0, b->n * sizeof(uint32_t));
        const int rc = cio_crc32_batch_host_multi((const void *const *) b->bufs, b->lens, b->seeds, out, b->n,
                                                  devs, ndev);
        CHECK(rc == 0 && same(out, b->want, b->n), "batch_host_multi ndev=%d rc=%d", ndev, rc);
    }
    free(out);
}

static void test_fd_multi(const struct batch *b, const char *dir)
{
    /* all chunks back to back in one file, at odd offsets */
    char path[4096];
    snprintf(path, sizeof(path), "%s/multi_chunks.bin", dir);
    const int fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0600);
    CHECK(fd >= 0, "open %s", path);
    if (fd < 0) {
        return;
    }
    uint64_t *foffs = calloc(b->n, sizeof(uint64_t));
    int *fds = calloc(b->n, sizeof(int));
    uint64_t at = 3;
    for (size_t i = 0; i < b->n; i++) {
        foffs[i] = at;
        fds[i] = fd;
        CHECK(pwrite(fd, b->bufs[i], b->lens[i], (off_t) at) == (ssize_t) b->lens[i], "pwrite");
        at += b->lens[i] + 7;
    }
    uint32_t *out = calloc(b->n, sizeof(uint32_t));
    for (int ndev = 1; ndev <= 3; ndev++) {
        memset(out, 0, b->n * sizeof(uint32_t));
        const int rc = cio_crc32_batch_fd_multi(fds, foffs, b->lens, b->seeds, out, b->n, devs, ndev);
        CHECK(rc == 0 && same(out, b->want, b->n), "batch_fd_multi ndev=%d rc=%d", ndev, rc);
    }
    /* a range past the end of the file is an error, not a wrong CRC */
    foffs[b->n - 1] = at + 100;
    size_t saved = b->lens[b->n - 1];
    b->lens[b->n - 1] = 10;
    CHECK(cio_crc32_batch_fd_multi(fds, foffs, b->lens, b->seeds, out, b->n, devs, 2) != 0, "short read");
    b->lens[b->n - 1] = saved;
    close(fd);
    unlink(path);
    free(out);
    free(fds);
    free(foffs);
}

static void test_split(void)
{
    const size_t sizes[] = {0, 1, 4095, 4096, 4097, 1000003, (64u << 20) + 12345};
    for (size_t s = 0; s < sizeof(sizes) / sizeof(sizes[0]); s++) {
        const size_t len = sizes[s];
        uint8_t *buf = malloc(len ? len : 1);
        for (size_t k = 0; k < len; k++) {
            buf[k] = (uint8_t) rng();
        }
        const uint32_t seed = s & 1 ? (uint32_t) rng() : 0xFFFFFFFFu;
        const uint32_t want = crc_bits(seed, buf, len);
        for (int ndev = 1; ndev <= 4; ndev++) {
            uint32_t got = 0;
            const int rc = cio_crc32_split_host_multi(buf, len, seed, &got, devs, ndev);
            CHECK(rc == 0 && got == want, "split len=%zu ndev=%d rc=%d got 0x%08x want 0x%08x", len, ndev, rc,
                  got, want);
        }
        free(buf);
    }
}

struct caller {
    const struct batch *b;
    int ndev;
    int ok;
};

static void *caller_main(void *arg)
{
    struct caller *c = arg;
    uint32_t *out = calloc(c->b->n, sizeof(uint32_t));
    c->ok = 1;
    for (int rep = 0; rep < 3; rep++) {
        memset(out, 0, c->b->n * sizeof(uint32_t));
        if (cio_crc32_batch_host_multi((const void *const *) c->b->bufs, c->b->lens, c->b->seeds, out, c->b->n,
                                       devs, c->ndev) != 0 ||
            memcmp(out, c->b->want, c->b->n * sizeof(uint32_t)) != 0) {
            c->ok = 0;
        }
    }
    free(out);
    return NULL;
}

/* 6 caller threads at once (more than the pool's 4 pipelines per device):
 * callers queue for an idle pipeline and every result stays exact. */
static void test_concurrent_callers(const struct batch *b)
{
    pthread_t th[6];
    struct caller c[6];
    for (int i = 0; i < 6; i++) {
        c[i].b = b;
        c[i].ndev = 1 + i % 3;
        pthread_create(&th[i], NULL, caller_main, &c[i]);
    }
    for (int i = 0; i < 6; i++) {
        pthread_join(th[i], NULL);
        CHECK(c[i].ok, "concurrent caller %d (ndev=%d)", i, c[i].ndev);
    }
}

int main(int argc, char **argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s <scratch dir>\n", argv[0]);
        return 2;
    }
    struct batch big, small;
    make_batch(&big, 61, 1);
    make_batch(&small, 200, 0);
    test_host_multi(&big);
    printf("%-24s %s\n", "host_multi", failures ? "FAILED" : "ok");
    fflush(stdout);
    int before = failures;
    test_fd_multi(&big, argv[1]);
    printf("%-24s %s\n", "fd_multi", failures != before ? "FAILED" : "ok");
    fflush(stdout);
    before = failures;
    test_split();
    printf("%-24s %s\n", "split_host_multi", failures != before ? "FAILED" : "ok");
    fflush(stdout);
    before = failures;
    test_concurrent_callers(&small);
    printf("%-24s %s\n", "concurrent_callers", failures != before ? "FAILED" : "ok");
    free_batch(&big);
    free_batch(&small);
    printf("multi: %d checks, %d failed\n", checks, failures);
    return failures ? 1 : 0;
}
