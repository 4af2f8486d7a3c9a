"""chunkio_amd -- MI355X-native replacement of fluent/chunkio's CRC-32
content-checksum path (and its SHA-1 content hash).

Layers:
  include/crc32/crc32.h, include/chunkio_amd/*.h   C ABI (the drop-in boundary)
  chunkio_amd/csrc/*.hip, *.c                      HIP kernels for gfx950 + host C
  chunkio_amd/crc32.py                             Python mirror of the CRC and SHA-1 API
                                                   (Sha1 / sha1_hash: chunkio's cio_sha1 on
                                                   OpenSSL-layout SHA_CTX bytes)
  chunkio_amd/chunkfile.py                         binding of the C chunk layer
                                                   (cioa_chunk.h: write/sync/verify/tx/scan,
                                                   up_batch)
"""
from ._lib import LIB_PATH, CioGpuError, lib  # noqa: F401
from .crc32 import (  # noqa: F401
    CRC_INIT, Crc32Plan, Crc32Ring, crc32, crc32_batch_cpu_packed, crc32_batch_dev, crc32_batch_host, crc32_batch_host_packed,
    crc32_combine, crc32_split_host, host_threads,
    crc32_shift, crc_finalize, crc_init, crc_update, device_count, fill_synthetic, host_register,
    host_unregister, pipe_last_timing, plan_cache_stats, split_rates, route, Sha1, sha1_hash, sha1_to_hex, sha1_batch_dev, sha1_batch_dev_async, sha1_final_batch_dev,
    sha1_states_init, sha1_states_view, sha1_update_batch_dev,
)

__version__ = "0.5.0"
