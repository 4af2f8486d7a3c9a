/*
 * cio_layout.h -- chunkio's on-disk chunk layout, host side (internal).
 *
 * include/chunkio/cio_file_st.h:116-179 and src/cio_file.c:45-60, 149-162 of
 * the reference, restated:
 *
 *   0..1   magic C1 00
 *   2..9   CRC: raw 8-byte crc_t state between a write and its sync,
 *          htonl(crc_finalize) in an 8-byte crc_t after the sync
 *   10..13 content length, big-endian u32
 *   22..23 metadata length, big-endian u16  <- the CRC region starts here
 *   24..   metadata, then content
 */
#ifndef CIOA_LAYOUT_H
#define CIOA_LAYOUT_H

#include <stdint.h>
#include <stddef.h>
#include <string.h>

#define CIOA_HDR_ID_00            0xc1
#define CIOA_HDR_ID_01            0x00
#define CIOA_HDR_MIN              24
#define CIOA_HDR_CONTENT_OFFSET   22
#define CIOA_HDR_CONTENT_LEN_OFF  10
/* crc_update(crc_init(), "\0\0", 2): crc_cur of a freshly initialised chunk */
#define CIOA_CRC_EMPTY_RAW        0xBE26ED00u

static inline uint16_t cioa_st_meta_len(const unsigned char *map)
{
    return (uint16_t) ((map[CIOA_HDR_CONTENT_OFFSET] << 8) | map[CIOA_HDR_CONTENT_OFFSET + 1]);
}

static inline void cioa_st_set_meta_len(unsigned char *map, uint16_t len)
{
    map[CIOA_HDR_CONTENT_OFFSET] = (unsigned char) (len >> 8);
    map[CIOA_HDR_CONTENT_OFFSET + 1] = (unsigned char) len;
}

static inline uint32_t cioa_st_get_content_len_field(const unsigned char *map)
{
    const unsigned char *b = map + CIOA_HDR_CONTENT_LEN_OFF;
    return ((uint32_t) b[0] << 24) | ((uint32_t) b[1] << 16) | ((uint32_t) b[2] << 8) | b[3];
}

static inline void cioa_st_set_content_len(unsigned char *map, uint32_t len)
{
    map[CIOA_HDR_CONTENT_LEN_OFF + 0] = (unsigned char) (len >> 24);
    map[CIOA_HDR_CONTENT_LEN_OFF + 1] = (unsigned char) (len >> 16);
    map[CIOA_HDR_CONTENT_LEN_OFF + 2] = (unsigned char) (len >> 8);
    map[CIOA_HDR_CONTENT_LEN_OFF + 3] = (unsigned char) len;
}

/* cio_file_st_get_content_len (cio_file_st.h:129-179), including the legacy
 * inference for files written before the length field existed (:166-176).
 * The reference writes the inferred length back unconditionally; here only
 * when the map is writable (writeback), since a read-only map cannot take
 * the store. */
static inline int64_t cioa_st_content_len(unsigned char *map, size_t size, int taint, int writeback)
{
    if (size < CIOA_HDR_MIN) {
        return -1;
    }
    const size_t content_offset = CIOA_HDR_CONTENT_OFFSET + 2 + cioa_st_meta_len(map);
    int64_t len = cioa_st_get_content_len_field(map);
    if (!taint && len == 0 && size > content_offset) {
        if (map[content_offset] != 0x00) {
            len = (int64_t) size - CIOA_HDR_MIN - cioa_st_meta_len(map);
            if (writeback) {
                cioa_st_set_content_len(map, (uint32_t) len);
            }
        }
    }
    return len;
}

/* write_init_header (cio_file.c:149-162) with cio_file_init_bytes (:45-60):
 * C1 00, ff 12 d9 41 (= LE 0x41D912FF), zero padding, meta_len 0; the CRC
 * bytes are zeroed when checksums are off; content length 0. */
static inline void cioa_write_init_header(unsigned char *map, int checksum)
{
    static const unsigned char init[CIOA_HDR_MIN] = {
        CIOA_HDR_ID_00, CIOA_HDR_ID_01, 0xff, 0x12, 0xd9, 0x41,
        0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    memcpy(map, init, sizeof(init));
    if (!checksum) {
        memset(map + 2, 0, 4);
    }
    cioa_st_set_content_len(map, 0);
}

#endif /* CIOA_LAYOUT_H */
