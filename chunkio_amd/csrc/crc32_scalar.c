/*
 * crc32_scalar.c -- the drop-in symbol `crc_update` declared by
 * include/crc32/crc32.h (replaces deps/crc32/crc32.c:337-390).
 */
#include <crc32/crc32.h>

#include "crc32_host.h"

crc_t crc_update(crc_t crc, const void *data, size_t data_len)
{
    return (crc_t) cioa_crc_update_host((uint64_t) crc, data, data_len);
}
