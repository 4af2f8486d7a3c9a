/*
 * cio_perf_port.c -- restatement of the reference's CPU perf-write path,
 * `tools/cio -k -p tests/data/400kb.txt` (BASELINE config 1).
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY (see crc32_oracle.c header).  It is
 * compiled twice by oracle/Makefile:
 *   - into oracle/liboracle_crc32.so with the oracle CRC      (kind "port")
 *   - into oracle/_ref/libcrc32_ref.so with the reference's own
 *     deps/crc32/crc32.c crc_update                            (kind "reference")
 * and is timed by bench.py's cpu_baseline leg on the GPU box's host cores.
 *
 * Per file it does what the reference does (file:line in fluent/chunkio):
 *   open O_RDWR|O_CREAT 0600                     src/cio_file_unix.c:396-417
 *   size = ROUND_UP(24, page); fallocate; mmap    src/cio_file.c:399-405, unix.c:100
 *   write init header (C1 00, ff 12 d9 41, ...)   src/cio_file.c:45-60, 149-162
 *   crc_cur = crc_update(init, map+22, 2)         src/cio_file.c:225 -> :92
 *   per write: grow alloc by realloc_size (8 pages) until it fits, page-round,
 *              fallocate + mremap(MAYMOVE)        src/cio_file.c:1025-1048
 *              crc_cur = crc_update(crc_cur, buf) src/cio_file.c:1058-1060, 97-113
 *              memcpy(map+2, &crc_cur, 8)         src/cio_file.c:111
 *              memcpy content; content_len (BE)   src/cio_file.c:1063-1068
 *   sync: htonl(~crc) as 8-byte crc_t -> map+2    src/cio_file.c:116-124, 1227
 *         msync(MS_ASYNC)                          src/cio_file_unix.c:477-497
 *   close: munmap; close                           src/cio_file.c:300-339
 * Timed region: the file loop only (tools/cio.c:411-434); bytes counted
 * exclude the 2-byte metadata-length prefix (tools/cio.c:424-430).
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stddef.h>
#include <stdio.h>
#include <string.h>
#include <errno.h>
#include <fcntl.h>
#include <unistd.h>
#include <time.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <arpa/inet.h>
#include <pthread.h>

#ifndef PORT_CRC_UPDATE
#error "define PORT_CRC_UPDATE to the crc_update implementation to time"
#endif
#ifndef PORT_PREFIX
#error "define PORT_PREFIX"
#endif

typedef uint_fast32_t port_crc_t;
extern port_crc_t PORT_CRC_UPDATE(port_crc_t crc, const void *data, size_t len);

#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)
#define PORT_FN(name) CAT(PORT_PREFIX, name)

#define HDR_MIN 24
#define ROUND_UP(N, S) ((((N) + (S) - 1) / (S)) * (S))

static const unsigned char init_bytes[HDR_MIN] = {
    0xc1, 0x00,                    /* file type */
    0xff, 0x12, 0xd9, 0x41,        /* crc32 of the 2-byte meta-length field */
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
    0x00, 0x00                     /* meta length */
};

static double now_sec(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return (double) ts.tv_sec + (double) ts.tv_nsec * 1e-9;
}

static void set_content_len(unsigned char *map, uint32_t len)
{
    map[10] = (unsigned char) (len >> 24);
    map[11] = (unsigned char) (len >> 16);
    map[12] = (unsigned char) (len >> 8);
    map[13] = (unsigned char) len;
}

static int grow(int fd, unsigned char **map, size_t *alloc, size_t new_size)
{
    void *tmp;
    if (fallocate(fd, 0, 0, (off_t) new_size) != 0) {
        if (errno != EOPNOTSUPP || posix_fallocate(fd, 0, (off_t) new_size) != 0) {
            return -1;
        }
    }
    tmp = mremap(*map, *alloc, new_size, MREMAP_MAYMOVE);
    if (tmp == MAP_FAILED) {
        return -1;
    }
    *map = (unsigned char *) tmp;
    *alloc = new_size;
    return 0;
}

/*
 * Run the perf-write loop.  Returns elapsed seconds (or -1 on error) and
 * the counted bytes in *bytes_out.  Files land in dir/perf-test-NNNN.txt.
 */
double PORT_FN(cio_perf_write)(const char *dir, const void *in_data, size_t in_size,
                               int files, int writes, int checksum,
                               uint64_t *bytes_out)
{
    char path[4096];
    size_t page = (size_t) sysconf(_SC_PAGESIZE);
    size_t realloc_size = page * 8;
    uint64_t bytes = 0;
    double t1, t2;

    t1 = now_sec();
    for (int i = 0; i < files; i++) {
        int fd;
        unsigned char *map;
        size_t alloc, data_size = 0;
        port_crc_t crc_cur = 0xffffffffu;

        snprintf(path, sizeof(path), "%s/perf-test-%04i.txt", dir, i);
        fd = open(path, O_RDWR | O_CREAT, 0600);
        if (fd < 0) {
            return -1.0;
        }
        alloc = ROUND_UP((size_t) HDR_MIN, page);
        if (fallocate(fd, 0, 0, (off_t) alloc) != 0 &&
            posix_fallocate(fd, 0, (off_t) alloc) != 0) {
            close(fd);
            return -1.0;
        }
        map = mmap(NULL, alloc, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (map == MAP_FAILED) {
            close(fd);
            return -1.0;
        }
        memcpy(map, init_bytes, HDR_MIN);
        if (!checksum) {
            map[2] = map[3] = map[4] = map[5] = 0;
        }
        set_content_len(map, 0);
        if (checksum) {
            crc_cur = PORT_CRC_UPDATE(crc_cur, map + 22, 2);
        }

        for (int j = 0; j < writes; j++) {
            size_t av = alloc - HDR_MIN - data_size;
            if (av < in_size) {
                size_t new_size = alloc + realloc_size;
                while (new_size < HDR_MIN + data_size + in_size) {
                    new_size += realloc_size;
                }
                new_size = ROUND_UP(new_size, page);
                if (grow(fd, &map, &alloc, new_size) != 0) {
                    munmap(map, alloc);
                    close(fd);
                    return -1.0;
                }
            }
            if (checksum) {
                crc_cur = PORT_CRC_UPDATE(crc_cur, in_data, in_size);
                memcpy(map + 2, &crc_cur, sizeof(crc_cur));
            }
            memcpy(map + HDR_MIN + data_size, in_data, in_size);
            data_size += in_size;
            set_content_len(map, (uint32_t) data_size);
            bytes += in_size;
        }

        if (checksum) {
            port_crc_t fin = htonl((uint32_t) (crc_cur ^ 0xffffffffu));
            memcpy(map + 2, &fin, sizeof(fin));
        }
        msync(map, alloc, MS_ASYNC);
        munmap(map, alloc);
        close(fd);
    }
    t2 = now_sec();
    if (bytes_out) {
        *bytes_out = bytes;
    }
    return t2 - t1;
}

/* CRC-only timing over a batch held in host RAM (one thread). */
double PORT_FN(crc_batch_time)(const unsigned char *base, const uint64_t *offs,
                               const uint64_t *lens, size_t n, int reps,
                               uint32_t *out)
{
    double t1 = now_sec();
    for (int r = 0; r < reps; r++) {
        for (size_t i = 0; i < n; i++) {
            out[i] = (uint32_t) PORT_CRC_UPDATE(0xffffffffu, base + offs[i], (size_t) lens[i]);
        }
    }
    return now_sec() - t1;
}

/* The same batch over `threads` host threads (chunk i -> thread i % threads),
 * for SURVEY §8(d)'s "1 thread and nproc threads" CPU figure. */
struct PORT_FN(mt_arg) {
    const unsigned char *base;
    const uint64_t *offs, *lens;
    size_t n, t, threads;
    int reps;
    uint32_t *out;
};

static void *PORT_FN(mt_worker)(void *p)
{
    struct PORT_FN(mt_arg) *a = p;
    for (int r = 0; r < a->reps; r++) {
        for (size_t i = a->t; i < a->n; i += a->threads) {
            a->out[i] = (uint32_t) PORT_CRC_UPDATE(0xffffffffu, a->base + a->offs[i], (size_t) a->lens[i]);
        }
    }
    return NULL;
}

double PORT_FN(crc_batch_time_mt)(const unsigned char *base, const uint64_t *offs,
                                  const uint64_t *lens, size_t n, int reps, int threads,
                                  uint32_t *out)
{
    pthread_t tid[256];
    struct PORT_FN(mt_arg) args[256];
    if (threads < 1) {
        threads = 1;
    }
    if (threads > 256) {
        threads = 256;
    }
    double t1 = now_sec();
    for (int t = 0; t < threads; t++) {
        args[t] = (struct PORT_FN(mt_arg)) {base, offs, lens, n, (size_t) t, (size_t) threads, reps, out};
        pthread_create(&tid[t], NULL, PORT_FN(mt_worker), &args[t]);
    }
    for (int t = 0; t < threads; t++) {
        pthread_join(tid[t], NULL);
    }
    return now_sec() - t1;
}
