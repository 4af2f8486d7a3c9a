"""Synthetic batch geometry and data for the BASELINE.json configurations.

Data generator (identical here, in the HIP fill kernel and in the tests):
    word_k(chunk i) = splitmix64(seed ^ (0x9E3779B97F4A7C15 * (i + 1)) + k)
emitted little-endian; chunk i is the first len_i bytes of word_0 word_1 ...
Uniform random bytes are the worst case for table-lookup CRC kernels.

Configs (BASELINE.json "configs"):
  2  1024 x 409,600 B, seed 0xC1000002                      (headline metric)
  3  65,536 chunks, len_i = floor(4096 * 1024**u_i),
     u_i = (splitmix64(0xC1000003 ^ i) >> 11) * 2**-53      (mixed 4 KB..4 MB)
  4  8192 x 4,194,304 B, seed 0xC1000004, chunk i -> GPU i mod G
  5  config-2 data, SHA-1
"""
import numpy as np

MASK64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15

CFG2_N, CFG2_LEN, CFG2_SEED = 1024, 409_600, 0xC1000002
CFG3_N, CFG3_SEED = 65_536, 0xC1000003
CFG4_N, CFG4_LEN, CFG4_SEED = 8192, 4 * 1024 * 1024, 0xC1000004
# 4 KiB records (the north star's small-chunk batch): cfg2's bytes in 4 KiB chunks
CFG4K_N, CFG4K_LEN, CFG4K_SEED = 102_400, 4096, 0xC1000006


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def chunk_key(seed, i):
    return (seed ^ ((GOLDEN * (i + 1)) & MASK64)) & MASK64


def gen_chunk(seed, i, length):
    """Bytes of chunk i (numpy uint8, length `length`)."""
    nwords = (length + 7) // 8
    with np.errstate(over="ignore"):
        k = np.arange(nwords, dtype=np.uint64) + np.uint64(chunk_key(seed, i))
    return splitmix64(k).view("<u8").view(np.uint8)[:length].copy()


def packed_offsets(lens, align=1, start=0):
    """Contiguous layout: offs[i] = start + sum(round_up(lens[:i], align))."""
    lens = np.asarray(lens, dtype=np.uint64)
    sizes = ((lens + np.uint64(align - 1)) // np.uint64(align)) * np.uint64(align)
    offs = np.zeros(len(lens), dtype=np.uint64)
    if len(lens) > 1:
        offs[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    return offs + np.uint64(start)


def batch_bytes(offs, lens):
    if len(offs) == 0:
        return 0
    return int((np.asarray(offs, np.uint64) + np.asarray(lens, np.uint64)).max())


def cfg2_lens(n=CFG2_N):
    return np.full(n, CFG2_LEN, dtype=np.uint64)


def cfg3_lens(n=CFG3_N, seed=CFG3_SEED):
    i = np.arange(n, dtype=np.uint64)
    u = (splitmix64(np.uint64(seed) ^ i) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
    return np.floor(4096.0 * np.power(1024.0, u)).astype(np.uint64)


def cfg4_lens(n=CFG4_N):
    return np.full(n, CFG4_LEN, dtype=np.uint64)


def shard_round_robin(n, rank, world):
    """Chunk indices owned by `rank` when chunk i goes to GPU i mod world."""
    return np.arange(rank, n, world, dtype=np.int64)


def host_batch(seed, lens, offs=None, align=1):
    """(buffer, offs) holding every chunk of a synthetic batch in host memory."""
    lens = np.asarray(lens, dtype=np.uint64)
    if offs is None:
        offs = packed_offsets(lens, align)
    buf = np.zeros(batch_bytes(offs, lens) + 16, dtype=np.uint8)
    for i, (o, ln) in enumerate(zip(offs, lens)):
        buf[int(o):int(o) + int(ln)] = gen_chunk(seed, i, int(ln))
    return buf, offs
