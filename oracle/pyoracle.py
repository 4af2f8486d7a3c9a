"""ctypes access to the oracle libraries -- TEST INFRASTRUCTURE ONLY.

  liboracle_crc32.so     C restatement of deps/crc32/crc32.c (crc32_oracle.c)
                         + the tools/cio perf-path port (kind "port")
  _ref/libcrc32_ref.so   the reference's own deps/crc32/crc32.c compiled from
                         /root/reference by oracle/Makefile (kind "reference");
                         prebuilt here, it travels to the GPU box with the repo.
SHA-1 oracle: hashlib (OpenSSL), FIPS 180-4 known answers in the tests, OpenSSL's
libcrypto for context bytes, and oracle/sha1_ctx.py (pure-Python SHA_CTX
restatement pinned to libcrypto) where libcrypto is not loadable.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle_crc32.so")
REF_SO = os.path.join(HERE, "_ref", "libcrc32_ref.so")

_oracle = None
_ref = None


def _ensure_built():
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)


def _bind_common(lib, prefix, crc_name):
    u64p = ctypes.POINTER(ctypes.c_uint64)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    f = getattr(lib, crc_name)
    f.restype = ctypes.c_uint64
    f.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t]
    f = getattr(lib, prefix + "cio_perf_write")
    f.restype = ctypes.c_double
    f.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                  ctypes.c_int, ctypes.c_int, u64p]
    f = getattr(lib, prefix + "crc_batch_time")
    f.restype = ctypes.c_double
    f.argtypes = [ctypes.c_void_p, u64p, u64p, ctypes.c_size_t, ctypes.c_int, u32p]
    return lib


def oracle():
    global _oracle
    if _oracle is None:
        _ensure_built()
        lib = _bind_common(ctypes.CDLL(ORACLE_SO), "oracle_", "oracle_crc_update")
        for name in ("oracle_crc_bitwise", "oracle_crc_shift", "oracle_crc_combine_raw"):
            getattr(lib, name).restype = ctypes.c_uint64
        lib.oracle_crc_bitwise.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t]
        lib.oracle_crc_shift.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        lib.oracle_crc_combine_raw.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        lib.oracle_multmodp.restype = ctypes.c_uint32
        lib.oracle_multmodp.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        lib.oracle_xpow8n.restype = ctypes.c_uint32
        lib.oracle_xpow8n.argtypes = [ctypes.c_uint64]
        lib.oracle_crc_batch.restype = None
        lib.oracle_crc_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                         ctypes.POINTER(ctypes.c_uint64),
                                         ctypes.POINTER(ctypes.c_uint32),
                                         ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t]
        _oracle = lib
    return _oracle


def ref():
    """The reference's compiled crc32.c, or None when it was never built."""
    global _ref
    if _ref is None and os.path.exists(REF_SO):
        _ref = _bind_common(ctypes.CDLL(REF_SO), "ref_", "crc_update")
    return _ref


def _buf(data):
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data).view(np.uint8)
    else:
        a = np.frombuffer(bytes(data), dtype=np.uint8)
    return a, (a.ctypes.data if a.size else None)


def crc_update(crc, data):
    a, p = _buf(data)
    return int(oracle().oracle_crc_update(crc, p, a.size))


def crc_update_ref(crc, data):
    lib = ref()
    if lib is None:
        raise RuntimeError("oracle/_ref/libcrc32_ref.so not built")
    a, p = _buf(data)
    return int(lib.crc_update(crc, p, a.size))


def crc_bitwise(crc, data):
    a, p = _buf(data)
    return int(oracle().oracle_crc_bitwise(crc, p, a.size))


def crc_shift(state, n):
    return int(oracle().oracle_crc_shift(state, n))


def crc_batch(buf, offs, lens, seeds=None):
    """Raw CRC states of every chunk of a host batch (numpy uint32)."""
    offs = np.ascontiguousarray(np.asarray(offs, dtype=np.uint64))
    lens = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64))
    out = np.zeros(len(offs), dtype=np.uint32)
    sp = None
    if seeds is not None:
        seeds = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint32))
        sp = seeds.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    oracle().oracle_crc_batch(buf.ctypes.data, offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                              lens.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), sp,
                              out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), len(offs))
    return out


def crc_batch_chunks(seed, lens, idx=None):
    """Raw CRC states (init seed) of synthetic chunks generated one at a time."""
    from chunkio_amd import workloads as wl   # generator only (pure numpy)
    lens = np.asarray(lens, dtype=np.uint64)
    idx = np.arange(len(lens)) if idx is None else np.asarray(idx)
    out = np.zeros(len(idx), dtype=np.uint32)
    for k, i in enumerate(idx):
        out[k] = crc_update(0xFFFFFFFF, wl.gen_chunk(seed, int(i), int(lens[int(i)])))
    return out
