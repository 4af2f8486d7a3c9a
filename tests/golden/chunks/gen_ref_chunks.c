/*
 * gen_ref_chunks.c -- writes tests/golden/chunks/ with the REFERENCE chunkio
 * (fluent/chunkio, built unmodified by its own CMake in /tmp by
 * tools/ref_dropin_ctest.sh; linked here against that build's
 * libchunkio-static.a + libcio-crc32.a).  Fixture generator only: nothing in
 * chunkio_amd/ or any GPU run builds or loads this file; make_ref_chunks.py
 * compiles and runs it in the build container.
 *
 * For each scenario it
 *   1. performs chunk operations through the reference API (cio_chunk_open,
 *      cio_meta_write, cio_chunk_write, cio_chunk_write_at, cio_chunk_sync,
 *      cio_chunk_close) in <out>/root/s/<name>, printing each operation as a
 *      JSON line so tests can replay exactly the same calls on chunkio_amd,
 *   2. optionally damages or rewrites the file the way a crash, a disk error
 *      or a pre-1.5 chunkio writer would (a "post" step, also printed),
 *   3. copies the final file to <out>/load/s/<name> and loads it the way
 *      cio_scan_stream_files does (src/cio_scan.c:102-105: cio_chunk_open
 *      with ctx->options.flags), printing the reference's verdict: err,
 *      ctx->last_chunk_error, and for a loaded chunk its crc_cur and content
 *      size.  The loaded copy is left as the reference's open + close left it
 *      (a legacy length is written back, src/cio_file.c:130-146 via
 *      cio_file_st.h:168-175).
 *
 * Content bytes are pattern(len, seed)[i] = ((i * 131 + seed * 7 + 17) % 251) + 1
 * (never 0, so the legacy-length inference sees a non-zero first byte).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chunkio/chunkio.h>
#include <chunkio/cio_chunk.h>
#include <chunkio/cio_file.h>
#include <chunkio/cio_meta.h>
#include <chunkio/cio_stream.h>

static const char *out_dir;
static FILE *man;
static int first_op;

static void die(const char *what)
{
    fprintf(stderr, "gen_ref_chunks: %s failed (%s)\n", what, strerror(errno));
    exit(1);
}

static void pattern(unsigned char *b, size_t len, int seed)
{
    for (size_t i = 0; i < len; i++) {
        b[i] = (unsigned char) (((i * 131u + (unsigned) seed * 7u + 17u) % 251u) + 1u);
    }
}

static void op_sep(void)
{
    fprintf(man, first_op ? "" : ", ");
    first_op = 0;
}

static struct cio_ctx *mk_ctx(const char *root, int flags)
{
    struct cio_options o;
    cio_options_init(&o);
    o.root_path = (char *) root;
    o.flags = flags;
    o.log_level = CIO_LOG_ERROR;
    struct cio_ctx *ctx = cio_create(&o);
    if (!ctx) {
        die("cio_create");
    }
    return ctx;
}

static void w(struct cio_chunk *ch, size_t len, int seed)
{
    unsigned char *b = malloc(len ? len : 1);
    pattern(b, len, seed);
    if (cio_chunk_write(ch, b, len) != 0) {
        die("cio_chunk_write");
    }
    free(b);
    op_sep();
    fprintf(man, "{\"op\": \"write\", \"len\": %zu, \"seed\": %d}", len, seed);
}

static void wat(struct cio_chunk *ch, size_t len, int seed, long off)
{
    unsigned char *b = malloc(len ? len : 1);
    pattern(b, len, seed);
    if (cio_chunk_write_at(ch, off, b, len) != 0) {
        die("cio_chunk_write_at");
    }
    free(b);
    op_sep();
    fprintf(man, "{\"op\": \"write_at\", \"len\": %zu, \"seed\": %d, \"offset\": %ld}", len, seed, off);
}

static void meta(struct cio_chunk *ch, const char *m)
{
    if (cio_meta_write(ch, (char *) m, strlen(m)) != 0) {
        die("cio_meta_write");
    }
    op_sep();
    fprintf(man, "{\"op\": \"meta_write\", \"meta\": \"%s\"}", m);
}

static void sync_(struct cio_chunk *ch)
{
    int rc = cio_chunk_sync(ch);
    op_sep();
    fprintf(man, "{\"op\": \"sync\", \"rc\": %d}", rc);
}

/* post-processing of the closed file: the damage each scenario models */
static void post_begin(void)
{
    fprintf(man, ", \"post\": [");
    first_op = 1;
}

static void post_end(void)
{
    fprintf(man, "]");
}

static void post_patch(const char *path, long off, const unsigned char *bytes, int n, const char *why)
{
    int fd = open(path, O_RDWR);
    if (fd < 0 || pwrite(fd, bytes, (size_t) n, off) != n) {
        die("patch");
    }
    close(fd);
    op_sep();
    fprintf(man, "{\"op\": \"patch\", \"offset\": %ld, \"hex\": \"", off);
    for (int i = 0; i < n; i++) {
        fprintf(man, "%02x", bytes[i]);
    }
    fprintf(man, "\", \"why\": \"%s\"}", why);
}

static void post_xor(const char *path, long off, unsigned char mask, const char *why)
{
    unsigned char b;
    int fd = open(path, O_RDWR);
    if (fd < 0 || pread(fd, &b, 1, off) != 1) {
        die("xor read");
    }
    b ^= mask;
    if (pwrite(fd, &b, 1, off) != 1) {
        die("xor write");
    }
    close(fd);
    op_sep();
    fprintf(man, "{\"op\": \"xor\", \"offset\": %ld, \"mask\": %u, \"why\": \"%s\"}", off, mask, why);
}

static void post_truncate(const char *path, off_t size, const char *why)
{
    if (truncate(path, size) != 0) {
        die("truncate");
    }
    op_sep();
    fprintf(man, "{\"op\": \"truncate\", \"size\": %lld, \"why\": \"%s\"}", (long long) size, why);
}

static void copy_file(const char *src, const char *dst)
{
    char buf[65536];
    int in = open(src, O_RDONLY), out = open(dst, O_WRONLY | O_CREAT | O_TRUNC, 0600);
    ssize_t n;
    if (in < 0 || out < 0) {
        die("copy open");
    }
    while ((n = read(in, buf, sizeof(buf))) > 0) {
        if (write(out, buf, (size_t) n) != n) {
            die("copy write");
        }
    }
    close(in);
    close(out);
}

/* cio_scan_stream_files' load of one file (src/cio_scan.c:102-105) */
static void load_verdict(const char *name, int flags)
{
    char root[4096], src[4096], dst[4096];
    snprintf(root, sizeof(root), "%s/load", out_dir);
    snprintf(src, sizeof(src), "%s/root/s/%s", out_dir, name);
    snprintf(dst, sizeof(dst), "%s/load/s/%s", out_dir, name);
    copy_file(src, dst);
    struct cio_ctx *ctx = mk_ctx(root, flags);
    struct cio_stream *st = cio_stream_create(ctx, "s", CIO_STORE_FS);
    int err = 0;
    ctx->last_chunk_error = 0;
    struct cio_chunk *ch = cio_chunk_open(ctx, st, name, ctx->options.flags, 0, &err);
    fprintf(man, ", \"load_flags\": %d, \"load\": {\"ok\": %s, \"err\": %d, \"last_chunk_error\": %d",
            flags, ch ? "true" : "false", err, ctx->last_chunk_error);
    if (ch) {
        struct cio_file *cf = (struct cio_file *) ch->backend;
        fprintf(man, ", \"crc_cur\": %lu, \"content_size\": %zd, \"meta_size\": %d",
                (unsigned long) cf->crc_cur, cio_chunk_get_content_size(ch), cio_meta_size(ch));
        cio_chunk_close(ch, CIO_FALSE);
    }
    fprintf(man, "}");
    cio_destroy(ctx);
}

enum { PLAIN, TRIM };

static struct cio_ctx *g_ctx;
static struct cio_stream *g_st, *g_st_trim;
static struct cio_ctx *g_ctx_trim;

static struct cio_chunk *begin(const char *name, int mode, size_t size)
{
    int err = 0;
    struct cio_chunk *ch = cio_chunk_open(mode == TRIM ? g_ctx_trim : g_ctx, mode == TRIM ? g_st_trim : g_st,
                                          name, CIO_OPEN, size, &err);
    if (!ch) {
        die("cio_chunk_open");
    }
    static int n_scen;
    fprintf(man, "%s{\"name\": \"%s\", \"ctx_flags\": %d, \"open_size\": %zu, \"ops\": [",
            n_scen++ ? ",\n " : "", name, (mode == TRIM ? g_ctx_trim : g_ctx)->options.flags, size);
    first_op = 1;
    return ch;
}

static const char *end(struct cio_chunk *ch, const char *name)
{
    static char path[4096];
    cio_chunk_close(ch, CIO_FALSE);
    op_sep();
    fprintf(man, "{\"op\": \"close\"}]");
    snprintf(path, sizeof(path), "%s/root/s/%s", out_dir, name);
    return path;
}

int main(int argc, char **argv)
{
    char root[4096], p[4096];
    const unsigned char zero4[4] = {0, 0, 0, 0};
    const unsigned char bad_magic[1] = {0xc2};
    struct cio_chunk *ch;
    const char *path;

    if (argc != 2) {
        fprintf(stderr, "usage: %s OUT_DIR   (writes OUT_DIR/root/s/*, OUT_DIR/load/s/*, manifest on stdout)\n",
                argv[0]);
        return 2;
    }
    out_dir = argv[1];
    snprintf(root, sizeof(root), "%s/root", out_dir);
    snprintf(p, sizeof(p), "%s/load", out_dir);
    if (mkdir(root, 0700) != 0 || mkdir(p, 0700) != 0) {
        die("mkdir (OUT_DIR must be empty)");
    }
    snprintf(p, sizeof(p), "%s/load/s", out_dir);
    if (mkdir(p, 0700) != 0) {
        die("mkdir load/s");
    }
    man = stdout;
    g_ctx = mk_ctx(root, CIO_CHECKSUM);
    g_st = cio_stream_create(g_ctx, "s", CIO_STORE_FS);
    g_ctx_trim = mk_ctx(root, CIO_CHECKSUM | CIO_TRIM_FILES);
    g_st_trim = cio_stream_create(g_ctx_trim, "s", CIO_STORE_FS);
    if (!g_st || !g_st_trim) {
        die("cio_stream_create");
    }
    fprintf(man, "[");

    /* an empty chunk, synced: header CRC 41 d9 12 ff (tests/fs.c:201-206) */
    ch = begin("c01_empty", PLAIN, 0);
    sync_(ch);
    end(ch, "c01_empty");
    load_verdict("c01_empty", CIO_CHECKSUM);
    fprintf(man, "}");

    /* content, no metadata */
    ch = begin("c02_content", PLAIN, 0);
    w(ch, 100, 1);
    w(ch, 37, 2);
    sync_(ch);
    end(ch, "c02_content");
    load_verdict("c02_content", CIO_CHECKSUM);
    fprintf(man, "}");

    /* metadata then content over a page and a realloc step, open size hint */
    ch = begin("c03_meta_content", PLAIN, 1000);
    meta(ch, "meta-abc");
    w(ch, 5000, 3);
    w(ch, 40000, 4);
    sync_(ch);
    end(ch, "c03_meta_content");
    load_verdict("c03_meta_content", CIO_CHECKSUM);
    fprintf(man, "}");

    /* write_at rewinds the content (src/cio_chunk.c:184-209), then appends */
    ch = begin("c04_write_at", PLAIN, 0);
    w(ch, 300, 5);
    w(ch, 200, 6);
    wat(ch, 150, 7, 120);
    w(ch, 50, 8);
    sync_(ch);
    end(ch, "c04_write_at");
    load_verdict("c04_write_at", CIO_CHECKSUM);
    fprintf(man, "}");

    /* metadata written after content: the content moves (adjust_layout,
     * src/cio_file.c:130-146) and the CRC is recomputed */
    ch = begin("c05_meta_after_content", PLAIN, 0);
    w(ch, 64, 9);
    meta(ch, "a-longer-metadata-block-0123456789-written-after-content");
    w(ch, 10, 10);
    meta(ch, "m2");
    sync_(ch);
    end(ch, "c05_meta_after_content");
    load_verdict("c05_meta_after_content", CIO_CHECKSUM);
    fprintf(man, "}");

    /* closed without an explicit sync (cio_chunk_close syncs) */
    ch = begin("c06_close_no_sync", PLAIN, 0);
    meta(ch, "x");
    w(ch, 4096, 11);
    end(ch, "c06_close_no_sync");
    load_verdict("c06_close_no_sync", CIO_CHECKSUM);
    fprintf(man, "}");

    /* a file cut to exactly 24 + meta + content whose content-length field
     * is zero: the layout a pre-1.5 chunkio wrote (no length at offset 10);
     * the loader infers the length from the file size (cio_file_st.h:160-175)
     * and writes it back */
    ch = begin("c07_legacy_exact", PLAIN, 0);
    meta(ch, "legacy");
    w(ch, 777, 12);
    sync_(ch);
    path = end(ch, "c07_legacy_exact");
    post_begin();
    post_patch(path, 10, zero4, 4, "pre-1.5 writer: no content length at offset 10");
    post_truncate(path, 24 + 6 + 777, "file exactly 24 + meta + content");
    post_end();
    load_verdict("c07_legacy_exact", CIO_CHECKSUM);
    fprintf(man, "}");

    /* the same on a page-padded file (CIO_TRIM_FILES rounds to a page): the
     * inferred length runs over the zero padding, so the CRC region differs */
    ch = begin("c08_legacy_padded", TRIM, 0);
    w(ch, 777, 12);
    sync_(ch);
    path = end(ch, "c08_legacy_padded");
    post_begin();
    post_patch(path, 10, zero4, 4, "content length zeroed on a page-padded file");
    post_end();
    load_verdict("c08_legacy_padded", CIO_CHECKSUM);
    fprintf(man, "}");

    /* truncated below its logical length (crash during a write) */
    ch = begin("c09_truncated", TRIM, 0);
    meta(ch, "meta-abc");
    w(ch, 5000, 3);
    sync_(ch);
    path = end(ch, "c09_truncated");
    post_begin();
    post_truncate(path, 24 + 8 + 5000 - 7, "file cut 7 bytes short of 24 + meta + content");
    post_end();
    load_verdict("c09_truncated", CIO_CHECKSUM);
    fprintf(man, "}");

    /* one flipped bit in the stored CRC */
    ch = begin("c10_bad_crc", PLAIN, 0);
    w(ch, 100, 1);
    w(ch, 37, 2);
    sync_(ch);
    path = end(ch, "c10_bad_crc");
    post_begin();
    post_xor(path, 3, 0x04, "one bit of the stored CRC flipped");
    post_end();
    load_verdict("c10_bad_crc", CIO_CHECKSUM);
    fprintf(man, "}");

    /* one flipped bit in the content */
    ch = begin("c11_bad_content", PLAIN, 0);
    meta(ch, "meta-abc");
    w(ch, 5000, 3);
    sync_(ch);
    path = end(ch, "c11_bad_content");
    post_begin();
    post_xor(path, 24 + 8 + 4321, 0x80, "one bit of the content flipped");
    post_end();
    load_verdict("c11_bad_content", CIO_CHECKSUM);
    fprintf(man, "}");

    /* bad magic */
    ch = begin("c12_bad_magic", PLAIN, 0);
    w(ch, 100, 1);
    sync_(ch);
    path = end(ch, "c12_bad_magic");
    post_begin();
    post_patch(path, 0, bad_magic, 1, "first byte not 0xc1");
    post_end();
    load_verdict("c12_bad_magic", CIO_CHECKSUM);
    fprintf(man, "}");

    /* shorter than the 24-byte header */
    ch = begin("c13_short_header", PLAIN, 0);
    w(ch, 100, 1);
    sync_(ch);
    path = end(ch, "c13_short_header");
    post_begin();
    post_truncate(path, 10, "file shorter than the 24-byte header");
    post_end();
    load_verdict("c13_short_header", CIO_CHECKSUM);
    fprintf(man, "}");

    /* a damaged file loaded with checksums off: only layout checks apply */
    ch = begin("c14_bad_crc_nochecksum", PLAIN, 0);
    w(ch, 100, 1);
    sync_(ch);
    path = end(ch, "c14_bad_crc_nochecksum");
    post_begin();
    post_xor(path, 3, 0x04, "stored CRC damaged, loaded without CIO_CHECKSUM");
    post_end();
    load_verdict("c14_bad_crc_nochecksum", 0);
    fprintf(man, "}");

    fprintf(man, "]\n");
    cio_destroy(g_ctx_trim);
    cio_destroy(g_ctx);
    return 0;
}
