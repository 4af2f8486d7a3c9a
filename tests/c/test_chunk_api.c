/*
 * The reference's own chunk-level tests, replayed in C through this repo's
 * cioa_* API (include/chunkio_amd/cioa_chunk.h) against libchunkio_amd.so:
 *
 *   tests/fs.c:56-175     fs_write            tests/fs.c:181-287   fs_checksum
 *   tests/fs.c:293-432    fs_up_down          tests/fs.c:435-480   issue_51
 *   tests/fs.c:482-523    issue_flb_2025      tests/fs.c:525-618   fs_size_chunks_up
 *   tests/fs.c:620-724    issue_write_at      tests/fs.c:727-803   fs_up_down_up_append
 *   tests/fs.c:805-841    deep_hierarchy      tests/fs.c:843-940   legacy_success/failure
 *   tests/fs.c:942-1103   metadata_unsigned_underflow
 *   tests/metadata_update.c:55-181  metadata_update_with_content
 *   tests/metadata_update.c:187-277 metadata_multiple_updates
 *
 * plus what those tests do not reach: transactions (src/cio_chunk.c:423-502),
 * CIO_TRIM_FILES (src/cio_file.c:1192-1224), CIO_FULL_SYNC, the batched scan
 * with CIO_DELETE_IRRECOVERABLE (src/cio_scan.c:107-118), and byte identity of
 * deferred-CRC chunks against the reference's per-write path.
 *
 * usage: test_chunk_api <400kb.txt> <scratch dir> <immediate|deferred>
 * Every verify (open/up/scan) runs the GPU batch, so this needs a GPU; run by
 * tests/test_c_api.py (-m gpu).  Exit 0 = all checks passed.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <unistd.h>
#include <arpa/inet.h>
#include <sys/stat.h>

#include <crc32/crc32.h>
#include "chunkio_amd/cioa_chunk.h"

static int failures, checks;
static const char *g_root;
static int g_mode;             /* 0 or CIOA_DEFERRED_CRC */
static char *in_data;
static size_t in_size;

#define TEST_CHECK(cond)                                                            \
    do {                                                                            \
        checks++;                                                                   \
        if (!(cond)) {                                                              \
            fprintf(stderr, "  FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);       \
            failures++;                                                             \
        }                                                                           \
    } while (0)

static char *read_file(const char *path, size_t *size)
{
    FILE *f = fopen(path, "rb");
    if (!f) {
        return NULL;
    }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *b = malloc((size_t) n + 1);
    if (b && fread(b, 1, (size_t) n, f) != (size_t) n) {
        free(b);
        b = NULL;
    }
    fclose(f);
    *size = (size_t) n;
    return b;
}

static void rm_rf(const char *path)
{
    char cmd[4200];
    snprintf(cmd, sizeof(cmd), "rm -rf '%s'", path);
    if (system(cmd) != 0) {
        fprintf(stderr, "cannot remove %s\n", path);
    }
}

static void env_path(char *out, size_t cap, const char *sub)
{
    snprintf(out, cap, "%s/%s", g_root, sub);
}

static cioa_ctx *ctx_new(const char *sub, int flags)
{
    char p[4096];
    env_path(p, sizeof(p), sub);
    rm_rf(p);
    return cioa_create(p, flags | ((flags & CIO_CHECKSUM) ? g_mode : 0));
}

static uint32_t hash_be(cioa_chunk *ch)
{
    uint32_t v;
    memcpy(&v, cioa_chunk_hash(ch), 4);
    return ntohl(v);
}

static unsigned char *slurp(const char *path, size_t *n)
{
    return (unsigned char *) read_file(path, n);
}

/* tests/fs.c:56-175 */
static void test_fs_write(void)
{
    int err;
    char tmp[255];
    cioa_ctx *ctx = ctx_new("fs", CIO_CHECKSUM);
    TEST_CHECK(ctx != NULL);
    TEST_CHECK(cioa_chunk_open(ctx, NULL, "invalid", 0, 0, &err) == NULL);
    TEST_CHECK(cioa_stream_create(ctx, "") == NULL);
    TEST_CHECK(cioa_stream_create(ctx, "/") == NULL);
    cioa_stream *st = cioa_stream_create(ctx, "test-write");
    TEST_CHECK(st != NULL);
    const int n_files = 100;
    for (int i = 0; i < n_files; i++) {
        int len = snprintf(tmp, sizeof(tmp), "api-test-%04i.txt", i);
        cioa_chunk *c = cioa_chunk_open(ctx, st, tmp, CIO_OPEN, 1000000, &err);
        TEST_CHECK(c != NULL);
        if (!c) {
            continue;
        }
        if (i >= CIOA_MAX_CHUNKS_UP) {
            TEST_CHECK(cioa_chunk_is_up(c) == 0);
            cioa_chunk_up_force(c);
        }
        cioa_chunk_write(c, in_data, in_size);
        cioa_chunk_write(c, in_data, in_size);
        cioa_meta_write(c, tmp, (size_t) len);
        cioa_chunk_write(c, in_data, in_size);
        cioa_chunk_write(c, in_data, in_size);
        cioa_chunk_write(c, in_data, in_size);
        TEST_CHECK(cioa_chunk_sync(c) == 0);
    }
    cioa_destroy(ctx);

    /* scan it back: every file verifies (CRC over meta + 5 x 400 KB) */
    char p[4096];
    env_path(p, sizeof(p), "fs");
    ctx = cioa_create(p, CIO_CHECKSUM | g_mode);
    cioa_set_max_chunks_up(ctx, 1000);
    st = cioa_scan_stream(ctx, "test-write", NULL);
    TEST_CHECK(st != NULL);
    cioa_chunk *arr[128];
    const size_t n = cioa_stream_chunks(st, arr, 128);
    TEST_CHECK(n == (size_t) n_files);
    for (size_t i = 0; i < n && i < 128; i++) {
        TEST_CHECK(cioa_chunk_is_up(arr[i]));
        TEST_CHECK(cioa_chunk_get_content_size(arr[i]) == (ssize_t) (5 * in_size));
        char *meta;
        int mlen;
        TEST_CHECK(cioa_meta_read(arr[i], &meta, &mlen) == 0 && mlen == 17 &&
                   memcmp(meta, "api-test-", 9) == 0);
    }
    cioa_destroy(ctx);
}

/* tests/fs.c:181-287 */
static void test_fs_checksum(void)
{
    int err;
    cioa_ctx *ctx = ctx_new("fs", CIO_CHECKSUM);
    cioa_stream *st = cioa_stream_create(ctx, "test-crc32");
    cioa_chunk *c = cioa_chunk_open(ctx, st, "test1.out", CIO_OPEN, 10, &err);
    TEST_CHECK(c != NULL);
    TEST_CHECK(cioa_chunk_hash(c) != NULL);
    /* before the sync: the init bytes ff 12 d9 41 (cio_file.c:49-50) */
    TEST_CHECK(memcmp(cioa_chunk_hash(c), "\xff\x12\xd9\x41", 4) == 0);
    cioa_chunk_sync(c);
    TEST_CHECK(hash_be(c) == 0x41D912FFu);                 /* crc32_test1 */
    cioa_chunk_write(c, in_data, in_size);
    cioa_chunk_sync(c);
    TEST_CHECK(hash_be(c) == 0x103CFA67u);                 /* crc32_test2 */
    TEST_CHECK(memcmp(cioa_chunk_hash(c) + 4, "\0\0\0\0", 4) == 0);   /* 8-byte crc_t */
    cioa_destroy(ctx);
}

/* tests/fs.c:293-432 */
static void test_fs_up_down(void)
{
    int err;
    char path[4096];
    struct stat sb;
    cioa_ctx *ctx = ctx_new("fs", CIO_CHECKSUM);
    cioa_stream *st = cioa_stream_create(ctx, "test-crc32");
    cioa_chunk *c = cioa_chunk_open(ctx, st, "test1.out", CIO_OPEN, 10, &err);
    TEST_CHECK(c != NULL);
    TEST_CHECK(cioa_chunk_is_up(c) == 1);
    TEST_CHECK(cioa_chunk_down(c) == 0);
    TEST_CHECK(cioa_chunk_is_up(c) == 0);
    TEST_CHECK(cioa_chunk_up(c) == 0);
    TEST_CHECK(cioa_chunk_is_up(c) == 1);
    cioa_chunk_sync(c);
    TEST_CHECK(hash_be(c) == 0x41D912FFu);
    cioa_chunk_write(c, in_data, in_size);
    cioa_chunk_sync(c);
    /* fs_size refreshed after the sync (fs.c:403-411) */
    env_path(path, sizeof(path), "fs/test-crc32/test1.out");
    TEST_CHECK(stat(path, &sb) == 0);
    TEST_CHECK(sb.st_size == cioa_chunk_get_real_size(c));
    TEST_CHECK(cioa_chunk_down(c) == 0);
    TEST_CHECK(cioa_chunk_up(c) == 0);
    TEST_CHECK(hash_be(c) == 0x103CFA67u);
    TEST_CHECK(cioa_chunk_crc_cur(c) == (uint32_t) crc_update(crc_update(crc_init(), "\0\0", 2), in_data, in_size));
    cioa_destroy(ctx);
}

/* tests/fs.c:435-480: a chunk truncated to 1 byte must not crash the load */
static void test_issue_51(void)
{
    int err;
    char path[4096];
    cioa_ctx *ctx = ctx_new("tmp51", 0);
    cioa_stream *st = cioa_stream_create(ctx, "test");
    cioa_chunk_open(ctx, st, "c", CIO_OPEN, 1000, &err);
    cioa_destroy(ctx);
    env_path(path, sizeof(path), "tmp51/test/c");
    int fd = open(path, O_WRONLY);
    TEST_CHECK(fd != -1);
    TEST_CHECK(ftruncate(fd, 1) == 0);
    close(fd);
    env_path(path, sizeof(path), "tmp51");
    ctx = cioa_create(path, 0);
    st = cioa_stream_create(ctx, "test");
    cioa_chunk *c = cioa_chunk_open(ctx, st, "c", CIO_OPEN, 1000, &err);
    TEST_CHECK(c == NULL && err == CIO_CORRUPTED);
    TEST_CHECK(cioa_last_chunk_error(ctx) == CIO_ERR_BAD_FILE_SIZE);
    cioa_destroy(ctx);
}

/* tests/fs.c:482-523 (and deep_hierarchy :805-841 with flags 0) */
static void write_down_up_loop(const char *sub, int flags, int iters)
{
    int err;
    const char line[] = "this is a test line\n";
    cioa_ctx *ctx = ctx_new(sub, flags);
    TEST_CHECK(ctx != NULL);
    cioa_stream *st = cioa_stream_create(ctx, "test");
    cioa_chunk *c = cioa_chunk_open(ctx, st, "c", CIO_OPEN, 1000, &err);
    TEST_CHECK(c != NULL);
    int bad = 0;
    for (int i = 0; i < iters && c; i++) {
        bad |= cioa_chunk_write(c, line, strlen(line)) != CIO_OK;
        bad |= cioa_chunk_down(c) != CIO_OK;
        bad |= cioa_chunk_up(c) != CIO_OK;
    }
    TEST_CHECK(!bad);
    TEST_CHECK(c && cioa_chunk_get_content_size(c) == (ssize_t) (iters * strlen(line)));
    cioa_destroy(ctx);
}

static void test_issue_flb_2025(void)
{
    write_down_up_loop("tmp2025", CIO_CHECKSUM, 1000);
}

static void test_deep_hierarchy(void)
{
    write_down_up_loop("tmp/deep/log/dir", 0, 1000);
}

/* tests/fs.c:525-618 */
static void test_fs_size_chunks_up(void)
{
    int err;
    char name[32];
    const char line[] = "this is a test line\n";
    cioa_ctx *ctx = ctx_new("fs", CIO_CHECKSUM);
    cioa_set_max_chunks_up(ctx, 50);
    cioa_stream *st = cioa_stream_create(ctx, "test_size_chunks_up");
    for (int i = 0; i < 100; i++) {
        snprintf(name, sizeof(name), "test-%i", i);
        cioa_chunk *c = cioa_chunk_open(ctx, st, name, CIO_OPEN, 1000, &err);
        TEST_CHECK(c != NULL);
        if (!c) {
            continue;
        }
        if (i < 50) {
            TEST_CHECK(cioa_chunk_is_up(c) == 1);
            TEST_CHECK(cioa_chunk_write(c, line, strlen(line)) == CIO_OK);
            TEST_CHECK(cioa_chunk_down(c) == CIO_OK);
            TEST_CHECK(cioa_chunk_is_up(c) == 0);
            TEST_CHECK(cioa_chunk_up(c) == CIO_OK);
        }
        else {
            TEST_CHECK(cioa_chunk_is_up(c) == 0);
        }
    }
    TEST_CHECK(cioa_stream_size_chunks_up(st) == 50 * strlen(line));
    TEST_CHECK(cioa_total_chunks_up(ctx) == 50);
    cioa_destroy(ctx);
}

/* tests/fs.c:620-724 */
static void test_issue_write_at(void)
{
    int err;
    const char line[] = "this is a test line\n";
    const size_t len = strlen(line);
    cioa_ctx *ctx = ctx_new("fs", CIO_CHECKSUM);
    cioa_set_max_chunks_up(ctx, 50);
    cioa_stream *st = cioa_stream_create(ctx, "test_write_at");
    cioa_chunk *c = cioa_chunk_open(ctx, st, "test", CIO_OPEN, 1000, &err);
    TEST_CHECK(c != NULL);
    TEST_CHECK(cioa_chunk_write(c, line, len) == CIO_OK);
    TEST_CHECK(cioa_chunk_write(c, line, len) == CIO_OK);
    TEST_CHECK(cioa_chunk_write(c, line, len) == CIO_OK);
    TEST_CHECK(cioa_chunk_write_at(c, (off_t) (len * 2), "test\n", 5) == CIO_OK);
    TEST_CHECK(cioa_chunk_down(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_up(c) == CIO_OK);
    void *buf;
    size_t sz;
    TEST_CHECK(cioa_chunk_get_content_copy(c, &buf, &sz) == CIO_OK);
    TEST_CHECK(sz == 2 * len + 5 && memcmp((char *) buf + 2 * len, "test\n", 5) == 0);
    free(buf);
    /* corrupt the running CRC, write a byte: the next up must fail */
    cioa_chunk_set_crc_cur(c, 10);
    cioa_chunk_write(c, "\0", 1);
    TEST_CHECK(cioa_chunk_down(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_up(c) == CIO_CORRUPTED);
    TEST_CHECK(cioa_error_get(c) == CIO_ERR_BAD_CHECKSUM);
    TEST_CHECK(cioa_chunk_hash(c) == NULL && cioa_chunk_is_up(c) == 0);
    cioa_destroy(ctx);
}

/* tests/fs.c:727-803 */
static void test_fs_up_down_up_append(void)
{
    int err;
    void *out;
    size_t sz;
    cioa_ctx *ctx = ctx_new("fs", CIO_CHECKSUM);
    cioa_stream *st = cioa_stream_create(ctx, "cio");
    cioa_chunk *c = cioa_chunk_open(ctx, st, "c", CIO_OPEN, 1000, &err);
    TEST_CHECK(c != NULL);
    TEST_CHECK(cioa_chunk_get_content_copy(c, &out, &sz) == CIO_OK);
    TEST_CHECK(memcmp(out, "", 1) == 0 && sz == 0);
    free(out);
    TEST_CHECK(cioa_chunk_write(c, "line 1\n", 7) == CIO_OK);
    TEST_CHECK(cioa_chunk_get_content_copy(c, &out, &sz) == CIO_OK);
    TEST_CHECK(memcmp(out, "line 1\n", 8) == 0 && sz == 7);
    free(out);
    TEST_CHECK(cioa_chunk_down(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_up(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_get_content_copy(c, &out, &sz) == CIO_OK);
    TEST_CHECK(memcmp(out, "line 1\n", 8) == 0 && sz == 7);
    free(out);
    TEST_CHECK(cioa_chunk_write(c, "line 2\n", 7) == CIO_OK);
    TEST_CHECK(cioa_chunk_down(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_up(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_get_content_copy(c, &out, &sz) == CIO_OK);
    TEST_CHECK(memcmp(out, "line 1\nline 2\n", 15) == 0 && sz == 14);
    free(out);
    cioa_destroy(ctx);
}

/* tests/fs.c:843-940 */
static void legacy_core(int trigger_checksum_error)
{
    int err;
    char path[4096];
    cioa_ctx *ctx = ctx_new("fs", CIO_CHECKSUM);
    cioa_stream *st = cioa_stream_create(ctx, "test-legacy");
    cioa_set_max_chunks_up(ctx, 1);
    cioa_chunk *c = cioa_chunk_open(ctx, st, "test_chunk", CIO_OPEN, 1000, &err);
    TEST_CHECK(c != NULL);
    TEST_CHECK(cioa_chunk_write(c, in_data, 128) == 0);
    TEST_CHECK(cioa_chunk_down(c) == CIO_OK);
    /* truncate_file(): zero the content-length field, resize to 128 + 24 (+1) */
    env_path(path, sizeof(path), "fs/test-legacy/test_chunk");
    int fd = open(path, O_RDWR);
    TEST_CHECK(fd >= 0);
    TEST_CHECK(pwrite(fd, "\0\0\0\0", 4, 10) == 4);
    TEST_CHECK(ftruncate(fd, 128 + 24 + (trigger_checksum_error ? 1 : 0)) == 0);
    close(fd);
    const int ret = cioa_chunk_up(c);
    if (trigger_checksum_error) {
        TEST_CHECK(ret != CIO_OK);
        TEST_CHECK(cioa_error_get(c) == CIO_ERR_BAD_CHECKSUM);
    }
    else {
        TEST_CHECK(ret == CIO_OK);
        TEST_CHECK(cioa_chunk_get_content_size(c) == 128);
        size_t n;
        unsigned char *raw = slurp(path, &n);
        TEST_CHECK(raw && raw[10] == 0 && raw[11] == 0 && raw[12] == 0 && raw[13] == 128);  /* written back */
        free(raw);
    }
    cioa_destroy(ctx);
}

static void test_legacy_success(void)
{
    legacy_core(0);
}

static void test_legacy_failure(void)
{
    legacy_core(1);
}

static void check_meta_content(cioa_chunk *c, const char *meta, const char *content, size_t clen)
{
    char *mb;
    int ml;
    void *cb;
    size_t cs;
    TEST_CHECK(cioa_meta_read(c, &mb, &ml) == CIO_OK);
    TEST_CHECK(ml == (int) strlen(meta) && memcmp(mb, meta, strlen(meta)) == 0);
    TEST_CHECK(cioa_chunk_get_content_copy(c, &cb, &cs) == CIO_OK);
    TEST_CHECK(cs == clen && memcmp(cb, content, clen) == 0);
    free(cb);
}

/* tests/fs.c:942-1103 */
static void test_metadata_unsigned_underflow(void)
{
    int err;
    const char *small = "small";
    const char *large = "this-is-a-very-large-metadata-string-that-would-cause-unsigned-underflow-in-old-code";
    const char *content = "test-content";
    cioa_ctx *ctx = ctx_new("fs", CIO_CHECKSUM);
    cioa_stream *st = cioa_stream_create(ctx, "test_stream_underflow");
    cioa_chunk *c = cioa_chunk_open(ctx, st, "test_chunk_underflow", CIO_OPEN, 100, &err);
    TEST_CHECK(c != NULL);
    TEST_CHECK(cioa_meta_write(c, small, strlen(small)) == CIO_OK);
    TEST_CHECK(cioa_chunk_write(c, content, strlen(content)) == CIO_OK);
    check_meta_content(c, small, content, strlen(content));
    TEST_CHECK(cioa_meta_write(c, large, strlen(large)) == CIO_OK);
    check_meta_content(c, large, content, strlen(content));
    TEST_CHECK(cioa_chunk_sync(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_down(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_up(c) == CIO_OK);
    check_meta_content(c, large, content, strlen(content));
    cioa_destroy(ctx);
}

/* tests/metadata_update.c:55-181 */
static void test_metadata_update_with_content(void)
{
    int err;
    const char *initial = "initial-metadata";
    const char *updated = "this-is-a-much-longer-metadata-string-that-will-require-content-to-be-moved";
    const char *content = "This is test content data that must be preserved when metadata is updated.";
    const char *more = " Additional content appended after metadata update.";
    char expect[512];
    cioa_ctx *ctx = ctx_new("meta", CIO_CHECKSUM);
    cioa_stream *st = cioa_stream_create(ctx, "test_stream");
    cioa_chunk *c = cioa_chunk_open(ctx, st, "test_chunk", CIO_OPEN, 1000, &err);
    TEST_CHECK(c != NULL);
    TEST_CHECK(cioa_meta_write(c, initial, strlen(initial)) == CIO_OK);
    TEST_CHECK(cioa_chunk_write(c, content, strlen(content)) == CIO_OK);
    TEST_CHECK(cioa_meta_write(c, updated, strlen(updated)) == CIO_OK);
    TEST_CHECK(cioa_chunk_write(c, more, strlen(more)) == CIO_OK);
    snprintf(expect, sizeof(expect), "%s%s", content, more);
    TEST_CHECK(cioa_chunk_sync(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_down(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_is_up(c) == 0);
    TEST_CHECK(cioa_chunk_up(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_is_up(c) == 1);
    check_meta_content(c, updated, expect, strlen(expect));
    cioa_destroy(ctx);
}

/* tests/metadata_update.c:187-277 */
static void test_metadata_multiple_updates(void)
{
    int err;
    const char *strs[] = {"small", "medium-sized-metadata",
                          "very-long-metadata-string-that-exceeds-previous-sizes", "tiny",
                          "another-medium-metadata-string"};
    const char *content = "Test content that must remain intact";
    cioa_ctx *ctx = ctx_new("meta", CIO_CHECKSUM);
    cioa_stream *st = cioa_stream_create(ctx, "test_stream");
    cioa_chunk *c = cioa_chunk_open(ctx, st, "test_chunk2", CIO_OPEN, 1000, &err);
    TEST_CHECK(c != NULL);
    TEST_CHECK(cioa_chunk_write(c, content, strlen(content)) == CIO_OK);
    for (int i = 0; i < 5; i++) {
        TEST_CHECK(cioa_meta_write(c, strs[i], strlen(strs[i])) == CIO_OK);
        check_meta_content(c, strs[i], content, strlen(content));
    }
    TEST_CHECK(cioa_chunk_sync(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_down(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_up(c) == CIO_OK);
    check_meta_content(c, strs[4], content, strlen(content));
    cioa_destroy(ctx);
}

/* ---- beyond the reference's tests -------------------------------------- */

/* The reference's transaction semantics (cio_chunk.c:423-502): rollback
 * restores crc_cur (as uint32) and data_size, not the header; a following
 * write overwrites from the restored size.  Compared with the CRC computed
 * here from the bytes the reference would have hashed. */
static void test_tx(void)
{
    int err;
    char path[4096];
    cioa_ctx *ctx = ctx_new("tx", CIO_CHECKSUM);
    cioa_stream *st = cioa_stream_create(ctx, "s");
    cioa_chunk *c = cioa_chunk_open(ctx, st, "t", CIO_OPEN, 0, &err);
    TEST_CHECK(c != NULL);
    TEST_CHECK(cioa_chunk_write(c, in_data, 1000) == 0);
    TEST_CHECK(cioa_chunk_tx_begin(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_tx_begin(c) == CIO_OK);            /* already active */
    TEST_CHECK(cioa_chunk_write(c, in_data + 1000, 5000) == 0);
    TEST_CHECK(cioa_chunk_tx_rollback(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_tx_rollback(c) == -1);              /* no tx */
    TEST_CHECK(cioa_chunk_get_content_size(c) == 1000);
    TEST_CHECK(cioa_chunk_write(c, in_data + 7000, 300) == 0);
    TEST_CHECK(cioa_chunk_tx_begin(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_write(c, in_data + 9000, 700) == 0);
    TEST_CHECK(cioa_chunk_tx_commit(c) == CIO_OK);
    /* expected: crc over "\0\0" + d[0:1000] + d[7000:7300] + d[9000:9700] */
    crc_t e = crc_update(crc_init(), "\0\0", 2);
    e = crc_update(e, in_data, 1000);
    e = crc_update(e, in_data + 7000, 300);
    e = crc_update(e, in_data + 9000, 700);
    TEST_CHECK(hash_be(c) == (uint32_t) crc_finalize(e));
    TEST_CHECK(cioa_chunk_crc_cur(c) == (uint32_t) e);
    /* a locked chunk refuses a transaction with CIO_RETRY */
    TEST_CHECK(cioa_chunk_lock(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_tx_begin(c) == CIO_RETRY);
    TEST_CHECK(cioa_chunk_lock(c) == CIO_ERROR);
    TEST_CHECK(cioa_chunk_unlock(c) == CIO_OK);
    /* rollback then sync with no write: the header's content length still
     * says 2000 (rollback does not rewrite it) but the CRC is of the
     * restored 2000 -> the reference's quirk: the reload fails verify */
    TEST_CHECK(cioa_chunk_tx_begin(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_write(c, in_data, 50) == 0);
    TEST_CHECK(cioa_chunk_tx_rollback(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_sync(c) == 0);
    TEST_CHECK(hash_be(c) == (uint32_t) crc_finalize(e));
    TEST_CHECK(cioa_chunk_down(c) == 0);
    TEST_CHECK(cioa_chunk_up(c) == CIO_CORRUPTED && cioa_error_get(c) == CIO_ERR_BAD_CHECKSUM);
    env_path(path, sizeof(path), "tx/s/t");
    size_t n;
    unsigned char *raw = slurp(path, &n);
    TEST_CHECK(raw && ((raw[10] << 24) | (raw[11] << 16) | (raw[12] << 8) | raw[13]) == 2050);
    free(raw);
    /* tx across a metadata rewrite: rollback keeps the new layout */
    c = cioa_chunk_open(ctx, st, "m", CIO_OPEN, 0, &err);
    TEST_CHECK(c != NULL);
    TEST_CHECK(cioa_chunk_write(c, in_data, 4000) == 0);
    TEST_CHECK(cioa_chunk_tx_begin(c) == CIO_OK);
    TEST_CHECK(cioa_meta_write(c, "meta!", 5) == 0);
    TEST_CHECK(cioa_chunk_write(c, in_data, 10) == 0);
    TEST_CHECK(cioa_chunk_tx_rollback(c) == CIO_OK);
    TEST_CHECK(cioa_chunk_write(c, in_data + 20000, 100) == 0);
    TEST_CHECK(cioa_chunk_sync(c) == 0);
    e = crc_update(crc_init(), "\0\0", 2);
    e = crc_update(e, in_data, 4000);
    e = crc_update(e, in_data + 20000, 100);
    TEST_CHECK(hash_be(c) == (uint32_t) crc_finalize(e));
    cioa_destroy(ctx);
}

/* CIO_TRIM_FILES (cio_file.c:1192-1224): the file shrinks to the page-rounded
 * logical size at sync; the bytes up to it are unchanged and verify. */
static void test_trim(void)
{
    int err;
    char path[4096];
    struct stat sb;
    cioa_ctx *ctx = ctx_new("trim", CIO_CHECKSUM | CIO_TRIM_FILES);
    cioa_stream *st = cioa_stream_create(ctx, "s");
    cioa_chunk *c = cioa_chunk_open(ctx, st, "t", CIO_OPEN, 0, &err);
    TEST_CHECK(c != NULL);
    TEST_CHECK(cioa_chunk_write(c, in_data, 5000) == 0);      /* grows to 36864 */
    env_path(path, sizeof(path), "trim/s/t");
    TEST_CHECK(stat(path, &sb) == 0 && sb.st_size == 36864);
    TEST_CHECK(cioa_chunk_sync(c) == 0);
    TEST_CHECK(stat(path, &sb) == 0 && sb.st_size == 8192);   /* ROUND_UP(24 + 5000, 4096) */
    TEST_CHECK(cioa_chunk_get_real_size(c) == 8192);
    TEST_CHECK(cioa_chunk_write(c, in_data, 100) == 0);
    TEST_CHECK(cioa_chunk_down(c) == 0);
    TEST_CHECK(stat(path, &sb) == 0 && sb.st_size == 8192);
    TEST_CHECK(cioa_chunk_up(c) == 0);
    TEST_CHECK(cioa_chunk_get_content_size(c) == 5100);
    cioa_destroy(ctx);
    /* without the flag the file keeps its allocation */
    ctx = ctx_new("trim", CIO_CHECKSUM);
    st = cioa_stream_create(ctx, "s");
    c = cioa_chunk_open(ctx, st, "t", CIO_OPEN, 0, &err);
    TEST_CHECK(cioa_chunk_write(c, in_data, 5000) == 0);
    TEST_CHECK(cioa_chunk_sync(c) == 0);
    TEST_CHECK(stat(path, &sb) == 0 && sb.st_size == 36864);
    cioa_destroy(ctx);
}

/* CIO_FULL_SYNC: same bytes, msync(MS_SYNC) */
static void test_full_sync(void)
{
    int err;
    cioa_ctx *ctx = ctx_new("full", CIO_CHECKSUM | CIO_FULL_SYNC);
    cioa_stream *st = cioa_stream_create(ctx, "s");
    cioa_chunk *c = cioa_chunk_open(ctx, st, "t", CIO_OPEN, 0, &err);
    TEST_CHECK(cioa_chunk_write(c, in_data, in_size) == 0);
    TEST_CHECK(cioa_chunk_sync(c) == 0);
    TEST_CHECK(hash_be(c) == 0x103CFA67u);
    cioa_destroy(ctx);
}

/* Batched sync: 64 chunks in one cioa_chunk_sync_batch, then a scan with
 * CIO_DELETE_IRRECOVERABLE over them after damaging some. */
static void test_sync_batch_and_scan(void)
{
    int err;
    char name[64], path[4096];
    cioa_ctx *ctx = ctx_new("scan", CIO_CHECKSUM);
    cioa_set_max_chunks_up(ctx, 256);
    cioa_stream *st = cioa_stream_create(ctx, "s");
    cioa_chunk *arr[64];
    for (int i = 0; i < 64; i++) {
        snprintf(name, sizeof(name), "c%02d.flb", i);
        arr[i] = cioa_chunk_open(ctx, st, name, CIO_OPEN, 0, &err);
        TEST_CHECK(arr[i] != NULL);
        if (i % 5 == 0) {
            cioa_meta_write(arr[i], name, strlen(name));
        }
        cioa_chunk_write(arr[i], in_data + i * 97, (size_t) (i * 3001) % 200000);
    }
    TEST_CHECK(cioa_chunk_sync_batch(arr, 64) == CIO_OK);
    uint32_t crc[64];
    for (int i = 0; i < 64; i++) {
        crc[i] = cioa_chunk_crc_cur(arr[i]);
    }
    cioa_destroy(ctx);
    /* damage: 7 -> flipped content byte, 11 -> bad magic, 13 -> truncated,
     * 17 -> not a chunk name (extension filter), 19 -> empty file */
    env_path(path, sizeof(path), "scan/s/c07.flb");
    int fd = open(path, O_RDWR);
    unsigned char byte = 0;
    TEST_CHECK(pread(fd, &byte, 1, 24 + 1000) == 1);
    byte ^= 0x20;
    TEST_CHECK(pwrite(fd, &byte, 1, 24 + 1000) == 1);
    close(fd);
    env_path(path, sizeof(path), "scan/s/c11.flb");
    fd = open(path, O_RDWR);
    TEST_CHECK(pwrite(fd, "\xc2", 1, 0) == 1);
    close(fd);
    env_path(path, sizeof(path), "scan/s/c13.flb");
    TEST_CHECK(truncate(path, 100) == 0);
    env_path(path, sizeof(path), "scan/s/c19.flb");
    TEST_CHECK(truncate(path, 0) == 0);
    char from[4096], to[4096];
    env_path(from, sizeof(from), "scan/s/c17.flb");
    env_path(to, sizeof(to), "scan/s/c17.txt");
    TEST_CHECK(rename(from, to) == 0);

    env_path(path, sizeof(path), "scan");
    ctx = cioa_create(path, CIO_CHECKSUM | CIO_DELETE_IRRECOVERABLE | g_mode);
    cioa_set_max_chunks_up(ctx, 256);
    st = cioa_scan_stream(ctx, "s", ".flb");
    TEST_CHECK(st != NULL);
    cioa_chunk *got[64];
    const size_t n = cioa_stream_chunks(st, got, 64);
    TEST_CHECK(n == 60);                 /* 64 - 3 corrupted - 1 filtered */
    for (size_t k = 0; k < n; k++) {
        const char *nm = cioa_chunk_name(got[k]);
        const int i = atoi(nm + 1);
        TEST_CHECK(cioa_chunk_is_up(got[k]));
        if (i == 19) {
            TEST_CHECK(cioa_chunk_crc_cur(got[k]) == (g_mode ? 0xffffffffu : 0xBE26ED00u));
        }
        else {
            TEST_CHECK(cioa_chunk_crc_cur(got[k]) == crc[i]);
        }
    }
    cioa_destroy(ctx);
    struct stat sb;
    env_path(path, sizeof(path), "scan/s/c07.flb");
    TEST_CHECK(stat(path, &sb) != 0);    /* BAD_CHECKSUM: deleted */
    env_path(path, sizeof(path), "scan/s/c11.flb");
    TEST_CHECK(stat(path, &sb) != 0);    /* BAD_LAYOUT: deleted */
    env_path(path, sizeof(path), "scan/s/c13.flb");
    TEST_CHECK(stat(path, &sb) != 0);    /* BAD_FILE_SIZE: deleted */
    env_path(path, sizeof(path), "scan/s/c17.txt");
    TEST_CHECK(stat(path, &sb) == 0);    /* not scanned: kept */
    /* with the budget smaller than the directory the rest stays down */
    env_path(path, sizeof(path), "scan");
    ctx = cioa_create(path, CIO_CHECKSUM | g_mode);
    cioa_set_max_chunks_up(ctx, 10);
    st = cioa_scan_stream(ctx, "s", ".flb");
    TEST_CHECK(cioa_stream_chunks(st, got, 64) == 60);
    TEST_CHECK(cioa_total_chunks_up(ctx) == 10);
    cioa_destroy(ctx);
}

/* Deferred and immediate chunks fed the same operations end byte-identical:
 * this program runs once per mode, the second run compares its files with
 * the first run's (kept under <scratch>/identity-<mode>). */
static void test_identity_corpus(void)
{
    int err;
    char name[64], path[4096];
    cioa_ctx *ctx = ctx_new(g_mode ? "identity-deferred" : "identity-immediate", CIO_CHECKSUM);
    cioa_set_max_chunks_up(ctx, 512);
    cioa_stream *st = cioa_stream_create(ctx, "s");
    uint64_t x = 0x9E3779B97F4A7C15ull;
    cioa_chunk *arr[200];
    for (int i = 0; i < 200; i++) {
        snprintf(name, sizeof(name), "c%03d", i);
        arr[i] = cioa_chunk_open(ctx, st, name, CIO_OPEN, 0, &err);
        for (int op = 0; op < 8; op++) {
            x ^= x << 13;
            x ^= x >> 7;
            x ^= x << 17;
            const int kind = (int) (x % 10);
            const size_t len = (size_t) ((x >> 8) % 60000) + 1;
            const size_t off = (size_t) ((x >> 24) % (in_size - len));
            if (kind == 0) {
                cioa_meta_write(arr[i], in_data + off, len % 300);
            }
            else if (kind == 1) {
                cioa_chunk_write_at(arr[i], (off_t) (cioa_chunk_get_content_size(arr[i]) / 2),
                                    in_data + off, len);
            }
            else if (kind == 2) {
                cioa_chunk_tx_begin(arr[i]);
            }
            else if (kind == 3) {
                cioa_chunk_tx_rollback(arr[i]);
            }
            else if (kind == 4 && (i & 1)) {
                cioa_chunk_sync(arr[i]);
            }
            else {
                cioa_chunk_write(arr[i], in_data + off, len);
            }
        }
    }
    TEST_CHECK(cioa_chunk_sync_batch(arr, 200) == CIO_OK);
    cioa_destroy(ctx);
    if (g_mode) {
        int diff = 0;
        for (int i = 0; i < 200; i++) {
            size_t n1, n2;
            snprintf(name, sizeof(name), "identity-deferred/s/c%03d", i);
            env_path(path, sizeof(path), name);
            unsigned char *a = slurp(path, &n1);
            snprintf(name, sizeof(name), "identity-immediate/s/c%03d", i);
            env_path(path, sizeof(path), name);
            unsigned char *b = slurp(path, &n2);
            if (!a || !b || n1 != n2 || memcmp(a, b, n1) != 0) {
                diff++;
                fprintf(stderr, "  identity: c%03d differs\n", i);
            }
            free(a);
            free(b);
        }
        TEST_CHECK(diff == 0);
    }
}

/* The `tools/cio -k -p` loop through the benchmark driver: 20 files, the
 * reference's perf-file header on every one; in deferred mode also with each
 * batch's CRC pass overlapping the next batch's writes. */
static void test_perf_driver(void)
{
    char path[4096];
    double secs;
    uint64_t bytes;
    for (int pipelined = 0; pipelined <= (g_mode ? 1 : 0); pipelined++) {
        env_path(path, sizeof(path), "perf");
        rm_rf(path);
        TEST_CHECK(cioa_bench_perf_write(path, in_data, in_size, 20, 5, 8,
                                         CIO_CHECKSUM | g_mode | (pipelined ? CIOA_BENCH_PIPELINED_SYNC : 0),
                                         &secs, &bytes) == CIO_OK);
        TEST_CHECK(bytes == 20 * 5 * in_size);
        for (int i = 0; i < 20; i++) {
            char name[128];
            size_t n;
            snprintf(name, sizeof(name), "perf/test-perf/perf-test-%04d.txt", i);
            env_path(path, sizeof(path), name);
            unsigned char *raw = slurp(path, &n);
            TEST_CHECK(raw && n == 2068480 &&
                       memcmp(raw, "\xc1\x00\x08\x87\x40\xe7\x00\x00\x00\x00\x00\x1f\x40\x00", 14) == 0);
            free(raw);
        }
    }
}

/* cioa_chunk_sync_batch_begin / _end: three groups of chunks, each group's
 * CRC pass running while the next group is written; a write to a held chunk
 * and a close of one finish their batch first.  The files and crc_cur equal
 * those of the same operations synced by cioa_chunk_sync_batch. */
static void test_sync_batch_async(void)
{
    int err;
    char name[64], path[4096];
    uint32_t want[60], got[60];
    for (int pass = 0; pass < 2; pass++) {
        cioa_ctx *ctx = ctx_new(pass ? "async-b" : "async-a", CIO_CHECKSUM);
        cioa_set_max_chunks_up(ctx, 256);
        cioa_stream *st = cioa_stream_create(ctx, "s");
        cioa_chunk *arr[60];
        cioa_sync_job *job[3] = {NULL, NULL, NULL};
        for (int g = 0; g < 3; g++) {
            for (int i = 20 * g; i < 20 * g + 20; i++) {
                snprintf(name, sizeof(name), "c%02d", i);
                arr[i] = cioa_chunk_open(ctx, st, name, CIO_OPEN, 0, &err);
                TEST_CHECK(arr[i] != NULL);
                if (i % 7 == 0) {
                    cioa_meta_write(arr[i], name, strlen(name));
                }
                cioa_chunk_write(arr[i], in_data + i * 131, (size_t) (i * 7919) % 300000 + 1);
            }
            if (pass == 0) {
                TEST_CHECK(cioa_chunk_sync_batch(arr + 20 * g, 20) == CIO_OK);
            }
            else {
                TEST_CHECK(cioa_chunk_sync_batch_begin(arr + 20 * g, 20, &job[g]) == CIO_OK && job[g]);
            }
        }
        /* a write to a held chunk (group 2) and a close (group 1) */
        TEST_CHECK(cioa_chunk_write(arr[45], "tail", 4) == 0);
        TEST_CHECK(cioa_chunk_sync(arr[45]) == 0);
        if (pass == 1) {
            cioa_chunk_close(arr[30], 0);
            for (int g = 0; g < 3; g++) {
                TEST_CHECK(cioa_chunk_sync_batch_end(job[g]) == CIO_OK);
            }
        }
        for (int i = 0; i < 60; i++) {     /* (held chunks' crc_cur is current after end) */
            (pass ? got : want)[i] = (pass && i == 30) ? want[30] : cioa_chunk_crc_cur(arr[i]);
        }
        cioa_destroy(ctx);
    }
    int diff = 0;
    for (int i = 0; i < 60; i++) {
        size_t n1, n2;
        snprintf(name, sizeof(name), "async-a/s/c%02d", i);
        env_path(path, sizeof(path), name);
        unsigned char *a = slurp(path, &n1);
        snprintf(name, sizeof(name), "async-b/s/c%02d", i);
        env_path(path, sizeof(path), name);
        unsigned char *b = slurp(path, &n2);
        if (!a || !b || n1 != n2 || memcmp(a, b, n1) != 0 || want[i] != got[i]) {
            diff++;
            fprintf(stderr, "  async: c%02d differs\n", i);
        }
        free(a);
        free(b);
    }
    TEST_CHECK(diff == 0);
}

/* cioa_scan_streams over a root of three streams (cio_scan_streams,
 * src/cio_scan.c:128-162), then cioa_chunk_close_stream on each: every chunk
 * comes back with its crc_cur, and closing keeps the files. */
static void test_scan_streams(void)
{
    int err;
    char name[64], path[4096];
    uint32_t crc[3][5];
    cioa_ctx *ctx = ctx_new("streams", CIO_CHECKSUM);
    cioa_set_max_chunks_up(ctx, 64);
    for (int s = 0; s < 3; s++) {
        snprintf(name, sizeof(name), "st%d", s);
        cioa_stream *st = cioa_stream_create(ctx, name);
        for (int i = 0; i < 5; i++) {
            snprintf(name, sizeof(name), "c%d.flb", i);
            cioa_chunk *c = cioa_chunk_open(ctx, st, name, CIO_OPEN, 0, &err);
            TEST_CHECK(c != NULL);
            cioa_chunk_write(c, in_data + s * 1000 + i, (size_t) (s * 5 + i) * 7001 + 1);
            TEST_CHECK(cioa_chunk_sync(c) == 0);
            crc[s][i] = cioa_chunk_crc_cur(c);
            TEST_CHECK(cioa_chunk_is_file(c) == 1);
            TEST_CHECK(cioa_chunk_get_content_end_pos(c) != 0);
        }
        cioa_chunk_close_stream(st);
        TEST_CHECK(cioa_stream_chunks(st, NULL, 0) == 0);
    }
    cioa_destroy(ctx);
    env_path(path, sizeof(path), "streams");
    ctx = cioa_create(path, CIO_CHECKSUM | g_mode);
    cioa_set_max_chunks_up(ctx, 64);
    TEST_CHECK(cioa_scan_streams(ctx, ".flb") == 0);
    for (int s = 0; s < 3; s++) {
        snprintf(name, sizeof(name), "st%d", s);
        cioa_stream *st = cioa_stream_get(ctx, name);
        TEST_CHECK(st != NULL);
        cioa_chunk *got[8];
        TEST_CHECK(st && cioa_stream_chunks(st, got, 8) == 5);
        for (int k = 0; st && k < 5; k++) {
            const int i = cioa_chunk_name(got[k])[1] - '0';
            TEST_CHECK(cioa_chunk_crc_cur(got[k]) == crc[s][i]);
        }
    }
    cioa_destroy(ctx);
}

/* ---- batched up (cioa_chunk_up_batch) ------------------------------------ */

/* n chunk files in <sub>/s, content of varied sizes; chunk k with k % 7 == 3
 * gets a flipped content byte on disk (BAD_CHECKSUM at its next verify). */
static void ub_build(const char *sub, int n, int seed)
{
    int err;
    char name[64];
    cioa_ctx *ctx = ctx_new(sub, CIO_CHECKSUM);
    cioa_stream *st = cioa_stream_create(ctx, "s");
    for (int i = 0; i < n; i++) {
        snprintf(name, sizeof(name), "c%03d", i);
        cioa_chunk *c = cioa_chunk_open(ctx, st, name, CIO_OPEN, 0, &err);
        TEST_CHECK(c != NULL);
        cioa_chunk_write(c, in_data + (seed * 131 + i) % 4096, (size_t) 1000 + (size_t) ((i * 7919 + seed) % 60000));
        TEST_CHECK(cioa_chunk_sync(c) == 0);
    }
    cioa_destroy(ctx);
    for (int i = 3; i < n; i += 7) {
        char path[4096];
        snprintf(name, sizeof(name), "%s/s/c%03d", sub, i);
        env_path(path, sizeof(path), name);
        int fd = open(path, O_RDWR);
        unsigned char b = 0;
        TEST_CHECK(fd >= 0 && pread(fd, &b, 1, 30) == 1);
        b ^= 0x40;
        TEST_CHECK(pwrite(fd, &b, 1, 30) == 1);
        close(fd);
    }
}

/* Open <sub> with max_chunks_up = max, scan, put every chunk down: *out
 * holds the stream's chunks (registered, all down). */
static cioa_ctx *ub_load_down(const char *sub, int max, cioa_chunk **out, size_t cap, size_t *n)
{
    char path[4096];
    env_path(path, sizeof(path), sub);
    cioa_ctx *ctx = cioa_create(path, CIO_CHECKSUM | g_mode);
    cioa_set_max_chunks_up(ctx, max);
    cioa_stream *st = cioa_scan_stream(ctx, "s", NULL);
    TEST_CHECK(st != NULL);
    *n = st ? cioa_stream_chunks(st, out, cap) : 0;
    for (size_t k = 0; k < *n && k < cap; k++) {
        if (cioa_chunk_is_up(out[k])) {
            cioa_chunk_down(out[k]);
        }
    }
    return ctx;
}

/* cioa_chunk_up_batch over chunks of two contexts interleaved (budgets 8 and
 * 5, damaged chunks among them, one chunk listed twice) against the same
 * cioa_chunk_up calls in order on copies of the files: every status, error
 * number, crc_cur and up state, and both contexts' counters, agree. */
static void test_up_batch(void)
{
    cioa_chunk *a[2][64], *b[2][64], *list[2][140];
    size_t na[2], nb[2], m[2] = {0, 0};
    int st[2][140];
    ub_build("ubA0", 40, 1);
    ub_build("ubB0", 30, 2);
    ub_build("ubA1", 40, 1);
    ub_build("ubB1", 30, 2);
    cioa_ctx *ca[2], *cb[2];
    for (int r = 0; r < 2; r++) {
        ca[r] = ub_load_down(r ? "ubA1" : "ubA0", 8, a[r], 64, &na[r]);
        cb[r] = ub_load_down(r ? "ubB1" : "ubB0", 5, b[r], 64, &nb[r]);
        /* scans dropped the damaged chunks they reached; the rest are down */
        for (size_t k = 0; k < na[r] || k < nb[r]; k++) {
            if (k < na[r]) list[r][m[r]++] = a[r][k];
            if (k < nb[r]) list[r][m[r]++] = b[r][k];
        }
        list[r][m[r]++] = a[r][2];
    }
    TEST_CHECK(m[0] == m[1] && na[0] > 20 && nb[0] > 15);
    for (size_t k = 0; k < m[0]; k++) {
        st[0][k] = cioa_chunk_up(list[0][k]);
    }
    TEST_CHECK(cioa_chunk_up_batch(list[1], m[1], st[1]) == CIO_ERROR);   /* not all came up */
    int diff = 0, up = 0;
    for (size_t k = 0; k < m[0]; k++) {
        const int u0 = cioa_chunk_is_up(list[0][k]), u1 = cioa_chunk_is_up(list[1][k]);
        if (st[0][k] != st[1][k] || u0 != u1 || cioa_error_get(list[0][k]) != cioa_error_get(list[1][k]) ||
            (u0 && cioa_chunk_crc_cur(list[0][k]) != cioa_chunk_crc_cur(list[1][k]))) {
            diff++;
            fprintf(stderr, "  up_batch: entry %zu differs (%d/%d)\n", k, st[0][k], st[1][k]);
        }
        up += st[1][k] == CIO_OK;
    }
    TEST_CHECK(diff == 0);
    TEST_CHECK(up == 13);
    TEST_CHECK(cioa_total_chunks_up(ca[0]) == cioa_total_chunks_up(ca[1]) && cioa_total_chunks_up(ca[1]) == 8);
    TEST_CHECK(cioa_total_chunks_up(cb[0]) == cioa_total_chunks_up(cb[1]) && cioa_total_chunks_up(cb[1]) == 5);
    TEST_CHECK(cioa_last_chunk_error(ca[0]) == cioa_last_chunk_error(ca[1]));
    TEST_CHECK(cioa_last_chunk_error(cb[0]) == cioa_last_chunk_error(cb[1]));
    TEST_CHECK(cioa_chunk_up_batch(NULL, 0, NULL) == CIO_OK);
    for (int r = 0; r < 2; r++) {
        cioa_destroy(ca[r]);
        cioa_destroy(cb[r]);
    }
}

struct test {
    const char *name;
    void (*fn)(void);
};

static const struct test tests[] = {
    {"fs_write", test_fs_write},
    {"fs_checksum", test_fs_checksum},
    {"fs_up_down", test_fs_up_down},
    {"fs_size_chunks_up", test_fs_size_chunks_up},
    {"issue_51", test_issue_51},
    {"issue_flb_2025", test_issue_flb_2025},
    {"issue_write_at", test_issue_write_at},
    {"fs_up_down_up_append", test_fs_up_down_up_append},
    {"fs_deep_hierachy", test_deep_hierarchy},
    {"legacy_success", test_legacy_success},
    {"legacy_failure", test_legacy_failure},
    {"metadata_unsigned_underflow", test_metadata_unsigned_underflow},
    {"metadata_update_with_content", test_metadata_update_with_content},
    {"metadata_multiple_updates", test_metadata_multiple_updates},
    {"tx", test_tx},
    {"trim", test_trim},
    {"full_sync", test_full_sync},
    {"sync_batch_and_scan", test_sync_batch_and_scan},
    {"identity_corpus", test_identity_corpus},
    {"perf_driver", test_perf_driver},
    {"sync_batch_async", test_sync_batch_async},
    {"scan_streams", test_scan_streams},
    {"up_batch", test_up_batch},
    {NULL, NULL},
};

int main(int argc, char **argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: %s <400kb.txt> <scratch dir> <immediate|deferred> [test]\n", argv[0]);
        return 2;
    }
    in_data = read_file(argv[1], &in_size);
    if (!in_data || in_size != 409600) {
        fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    g_root = argv[2];
    g_mode = strcmp(argv[3], "deferred") == 0 ? CIOA_DEFERRED_CRC : 0;
    int failed_tests = 0;
    for (const struct test *t = tests; t->name; t++) {
        if (argc > 4 && strcmp(argv[4], t->name) != 0) {
            continue;
        }
        const int before = failures;
        t->fn();
        printf("%-32s %s\n", t->name, failures == before ? "ok" : "FAILED");
        fflush(stdout);
        failed_tests += failures != before;
    }
    printf("%s mode: %d checks, %d failed, %d test(s) failed\n", argv[3], checks, failures, failed_tests);
    free(in_data);
    return failures ? 1 : 0;
}
