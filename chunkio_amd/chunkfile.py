"""Python binding of the C chunk layer (include/chunkio_amd/cioa_chunk.h).

The chunk layer itself is C (chunkio_amd/csrc/cioa_chunk.c): chunkio's
filesystem backend with the reference's on-disk format and CRC lifecycle,
its verifies and deferred CRCs on the batched GPU path.  Names follow the
reference (file:line citations into /root/reference):

  Context(root, flags)            cio_create (src/chunkio.c:84-207)
  Context.stream(name)            cio_stream_create (src/cio_stream.c:113-178)
  Context.scan(stream, ext)       cio_scan_stream_files (src/cio_scan.c:39-125), one
                                  GPU verify batch, CIO_DELETE_IRRECOVERABLE
  Stream.open(name, flags)        cio_chunk_open (src/cio_chunk.c:30-109)
  Chunk.write / write_at          cio_chunk_write / _write_at (src/cio_chunk.c:184-227)
  Chunk.meta_write / meta_len     cio_meta_write / _size (src/cio_meta.c:46-88)
  Chunk.sync / sync_batch(chunks) cio_chunk_sync (src/cio_file.c:1147-1250); batched
  Chunk.up / up_force / down      src/cio_chunk.c:556-605
  Chunk.tx_begin/commit/rollback  src/cio_chunk.c:423-502
  Chunk.hash()                    cio_chunk_hash: the 4 bytes at map+2

ChunkFile.open(path, ...) is the one-chunk convenience form used by the
tests and benches: a private context rooted at dirname(dirname(path)) with
the stream dirname(path).

verify_paths(paths) is the batched verify-on-load of a list of chunk files
(cio_verify_paths_multi).
"""
import ctypes
import os
import struct

import numpy as np

from . import _lib

CIO_OK, CIO_ERROR, CIO_RETRY, CIO_CORRUPTED = 0, -1, -2, -3
CIO_OPEN, CIO_OPEN_RD, CIO_CHECKSUM, CIO_FULL_SYNC = 1, 2, 4, 8
CIO_DELETE_IRRECOVERABLE, CIO_TRIM_FILES = 16, 32
CIOA_DEFERRED_CRC = 128
CIOA_BENCH_PIPELINED_SYNC = 0x10000      # cioa_bench_perf_write only
CIO_ERR_BAD_CHECKSUM, CIO_ERR_BAD_LAYOUT, CIO_ERR_PERMISSION, CIO_ERR_BAD_FILE_SIZE = -10, -11, -12, -13
CIOA_VERIFY_DELETE_IRRECOVERABLE = 16
CIOA_VERIFY_WRITEBACK = 64
CIOA_SYNC_FINALIZE, CIOA_SYNC_MSYNC, CIOA_SYNC_FULL = 1, 2, 8

HDR_MIN = 24
CONTENT_OFFSET = 22
CRC_INIT = 0xFFFFFFFF


class VerifyItem(ctypes.Structure):
    _fields_ = [("map", ctypes.c_void_p), ("fs_size", ctypes.c_size_t), ("taint", ctypes.c_int),
                ("status", ctypes.c_int), ("error", ctypes.c_int), ("crc_raw", ctypes.c_uint32),
                ("meta_len", ctypes.c_uint16), ("content_len", ctypes.c_uint64)]


class SyncItem(ctypes.Structure):
    _fields_ = [("map", ctypes.c_void_p), ("fs_size", ctypes.c_size_t), ("crc_end", ctypes.c_uint64),
                ("crc_cur", ctypes.c_uint32), ("status", ctypes.c_int), ("data_end", ctypes.c_uint64)]


def _bind():
    lib = _lib.lib()
    if getattr(lib, "_chunk_bound", False):
        return lib
    V, I, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    IP, U32 = ctypes.POINTER(ctypes.c_int), ctypes.c_uint32
    sig = {
        "cio_file_verify_batch": (I, [ctypes.POINTER(VerifyItem), S, I]),
        "cio_file_verify_batch_multi": (I, [ctypes.POINTER(VerifyItem), S, I, IP, I]),
        "cio_verify_paths": (I, [ctypes.POINTER(ctypes.c_char_p), S, I, IP, IP, ctypes.POINTER(U32)]),
        "cio_verify_paths_multi": (I, [ctypes.POINTER(ctypes.c_char_p), S, I, IP, I, IP, IP,
                                       ctypes.POINTER(U32)]),
        "cio_file_sync_batch": (I, [ctypes.POINTER(SyncItem), S, I]),
        "cio_file_sync_batch_multi": (I, [ctypes.POINTER(SyncItem), S, I, IP, I]),
        "cioa_create": (V, [ctypes.c_char_p, I]),
        "cioa_destroy": (None, [V]),
        "cioa_set_max_chunks_up": (I, [V, I]),
        "cioa_set_realloc_size_hint": (I, [V, S]),
        "cioa_set_devices": (I, [V, IP, I]),
        "cioa_last_chunk_error": (I, [V]),
        "cioa_total_chunks_up": (S, [V]),
        "cioa_stream_create": (V, [V, ctypes.c_char_p]),
        "cioa_stream_get": (V, [V, ctypes.c_char_p]),
        "cioa_stream_chunks": (S, [V, ctypes.POINTER(V), S]),
        "cioa_stream_size_chunks_up": (S, [V]),
        "cioa_scan_stream": (V, [V, ctypes.c_char_p, ctypes.c_char_p]),
        "cioa_scan_streams": (I, [V, ctypes.c_char_p]),
        "cioa_scan_dump": (I, [V, V]),
        "cioa_chunk_open": (V, [V, V, ctypes.c_char_p, I, S, IP]),
        "cioa_chunk_close": (None, [V, I]),
        "cioa_chunk_write": (I, [V, V, S]),
        "cioa_chunk_write_at": (I, [V, ctypes.c_long, V, S]),
        "cioa_chunk_sync": (I, [V]),
        "cioa_chunk_sync_batch": (I, [ctypes.POINTER(V), S]),
        "cioa_chunk_sync_batch_begin": (I, [ctypes.POINTER(V), S, ctypes.POINTER(V)]),
        "cioa_chunk_sync_batch_end": (I, [V]),
        "cio_file_sync_batch_begin": (I, [ctypes.POINTER(SyncItem), S, I, IP, I, ctypes.POINTER(V)]),
        "cio_file_sync_batch_end": (I, [V]),
        "cioa_chunk_get_content_size": (ctypes.c_ssize_t, [V]),
        "cioa_chunk_get_content_end_pos": (S, [V]),
        "cioa_chunk_is_file": (I, [V]),
        "cioa_chunk_close_stream": (None, [V]),
        "cioa_chunk_get_real_size": (ctypes.c_ssize_t, [V]),
        "cioa_chunk_hash": (V, [V]),
        "cioa_chunk_map": (V, [V, ctypes.POINTER(S)]),
        "cioa_chunk_name": (ctypes.c_char_p, [V]),
        "cioa_chunk_lock": (I, [V]),
        "cioa_chunk_unlock": (I, [V]),
        "cioa_chunk_tx_begin": (I, [V]),
        "cioa_chunk_tx_commit": (I, [V]),
        "cioa_chunk_tx_rollback": (I, [V]),
        "cioa_chunk_is_up": (I, [V]),
        "cioa_chunk_up": (I, [V]),
        "cioa_chunk_up_force": (I, [V]),
        "cioa_chunk_up_batch": (I, [ctypes.POINTER(V), S, IP]),
        "cioa_chunk_up_force_batch": (I, [ctypes.POINTER(V), S, IP]),
        "cioa_chunk_down": (I, [V]),
        "cioa_error_get": (I, [V]),
        "cioa_chunk_crc_cur": (U32, [V]),
        "cioa_chunk_set_crc_cur": (None, [V, U32]),
        "cioa_meta_write": (I, [V, ctypes.c_char_p, S]),
        "cioa_meta_size": (I, [V]),
        "cioa_bench_perf_write": (I, [ctypes.c_char_p, V, S, I, I, I, I, ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_uint64)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    lib._chunk_bound = True
    return lib


def _devs(devices):
    if not devices:
        return None, 0
    arr = (ctypes.c_int * len(devices))(*devices)
    return arr, len(devices)


def verify_paths(paths, flags=CIO_CHECKSUM, devices=None):
    """Batched verify-on-load: (status, error, crc_raw) numpy arrays per path."""
    lib = _bind()
    n = len(paths)
    arr = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(p) for p in paths])
    st = np.zeros(max(n, 1), np.int32)
    er = np.zeros(max(n, 1), np.int32)
    cr = np.zeros(max(n, 1), np.uint32)
    dv, nd = _devs(devices)
    rc = lib.cio_verify_paths_multi(arr, n, flags, dv, nd, st.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                    er.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                    cr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    _lib.check(rc, "cio_verify_paths_multi")
    return st[:n], er[:n], cr[:n]


class Context:
    """cio_ctx: a root directory of streams of chunk files."""

    def __init__(self, root, flags=CIO_CHECKSUM, devices=None, max_chunks_up=None):
        self._lib = _bind()
        self.root = root
        self._h = self._lib.cioa_create(os.fsencode(root), flags)
        if not self._h:
            raise OSError(f"cioa_create({root!r}) failed")
        if devices:
            dv, nd = _devs(devices)
            self._lib.cioa_set_devices(self._h, dv, nd)
        if max_chunks_up is not None:
            self._lib.cioa_set_max_chunks_up(self._h, int(max_chunks_up))
        self._chunks = []

    def stream(self, name):
        h = self._lib.cioa_stream_get(self._h, name.encode()) or self._lib.cioa_stream_create(self._h, name.encode())
        if not h:
            raise OSError(f"cannot create stream {name!r}")
        return Stream(self, h, name)

    def scan(self, stream, ext=None):
        """Load a stream directory (one batched GPU verify): (Stream, [Chunk])."""
        h = self._lib.cioa_scan_stream(self._h, stream.encode(), ext.encode() if ext else None)
        if not h:
            raise OSError(f"cannot scan stream {stream!r}")
        st = Stream(self, h, stream)
        return st, st.chunks()

    def scan_all(self, ext=None):
        """cioa_scan_streams: load every stream directory of the root (the
        verifies of all streams batched together): {stream name: [Chunk]}."""
        if self._lib.cioa_scan_streams(self._h, ext.encode() if ext else None) != 0:
            raise OSError("cannot scan the root")
        out = {}
        for name in sorted(os.listdir(self.root)):
            h = self._lib.cioa_stream_get(self._h, name.encode())
            if h:
                out[name] = Stream(self, h, name).chunks()
        return out

    def dump(self):
        """The `tools/cio -l` listing of every stream (cioa_scan_dump), as text."""
        import tempfile
        libc = ctypes.CDLL(None)
        libc.fopen.restype = ctypes.c_void_p
        libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        libc.fclose.argtypes = [ctypes.c_void_p]
        with tempfile.NamedTemporaryFile(prefix="cioa-dump-") as tf:
            fp = libc.fopen(tf.name.encode(), b"w")
            if not fp:
                raise OSError("fopen failed")
            try:
                rc = self._lib.cioa_scan_dump(self._h, fp)
            finally:
                libc.fclose(fp)
            if rc != 0:
                raise OSError("cioa_scan_dump failed")
            with open(tf.name, "r") as f:
                return f.read()

    @property
    def last_chunk_error(self):
        return int(self._lib.cioa_last_chunk_error(self._h))

    @property
    def total_chunks_up(self):
        return int(self._lib.cioa_total_chunks_up(self._h))

    def close(self):
        if self._h:
            for c in self._chunks:
                c._h = None
            self._lib.cioa_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class Stream:
    def __init__(self, ctx, h, name):
        self.ctx, self._h, self.name = ctx, h, name

    def open(self, name, flags=CIO_OPEN, size=0):
        """(Chunk or None, err)."""
        err = ctypes.c_int(0)
        h = self.ctx._lib.cioa_chunk_open(self.ctx._h, self._h, name.encode(), flags, size, ctypes.byref(err))
        if not h:
            return None, int(err.value)
        c = Chunk(self.ctx, h)
        self.ctx._chunks.append(c)
        return c, CIO_OK

    def chunks(self):
        lib = self.ctx._lib
        n = int(lib.cioa_stream_chunks(self._h, None, 0))
        arr = (ctypes.c_void_p * max(n, 1))()
        lib.cioa_stream_chunks(self._h, arr, n)
        known = {c._h: c for c in self.ctx._chunks if c._h}
        out = []
        for i in range(n):
            c = known.get(arr[i])
            if c is None:
                c = Chunk(self.ctx, arr[i])
                self.ctx._chunks.append(c)
            out.append(c)
        return out

    def size_chunks_up(self):
        return int(self.ctx._lib.cioa_stream_size_chunks_up(self._h))

    def close_chunks(self):
        """cioa_chunk_close_stream: close every chunk of the stream (files kept)."""
        chunks = self.chunks()
        self.ctx._lib.cioa_chunk_close_stream(self._h)
        for c in chunks:
            c._h = None


class Chunk:
    """cio_chunk over the C layer."""

    def __init__(self, ctx, h):
        self.ctx, self._h, self._lib = ctx, h, ctx._lib

    def _c(self):
        if not self._h:
            raise ValueError("chunk is closed")
        return self._h

    @property
    def name(self):
        return self._lib.cioa_chunk_name(self._c()).decode()

    def write(self, data):
        b = bytes(data)
        return int(self._lib.cioa_chunk_write(self._c(), b, len(b)))

    def write_at(self, data, offset):
        b = bytes(data)
        return int(self._lib.cioa_chunk_write_at(self._c(), int(offset), b, len(b)))

    def meta_write(self, meta):
        b = bytes(meta)
        return int(self._lib.cioa_meta_write(self._c(), b, len(b)))

    write_metadata = meta_write

    def meta_len(self):
        return int(self._lib.cioa_meta_size(self._c()))

    def sync(self):
        return int(self._lib.cioa_chunk_sync(self._c()))

    def up(self):
        return int(self._lib.cioa_chunk_up(self._c()))

    def up_force(self):
        return int(self._lib.cioa_chunk_up_force(self._c()))

    def down(self):
        return int(self._lib.cioa_chunk_down(self._c()))

    def is_up(self):
        return bool(self._lib.cioa_chunk_is_up(self._c()))

    def lock(self):
        return int(self._lib.cioa_chunk_lock(self._c()))

    def unlock(self):
        return int(self._lib.cioa_chunk_unlock(self._c()))

    def tx_begin(self):
        return int(self._lib.cioa_chunk_tx_begin(self._c()))

    def tx_commit(self):
        return int(self._lib.cioa_chunk_tx_commit(self._c()))

    def tx_rollback(self):
        return int(self._lib.cioa_chunk_tx_rollback(self._c()))

    @property
    def error(self):
        return int(self._lib.cioa_error_get(self._c()))

    @property
    def data_size(self):
        return int(self._lib.cioa_chunk_get_content_size(self._c()))

    @property
    def content_end_pos(self):
        return int(self._lib.cioa_chunk_get_content_end_pos(self._c()))

    def is_file(self):
        return bool(self._lib.cioa_chunk_is_file(self._c()))

    @property
    def real_size(self):
        return int(self._lib.cioa_chunk_get_real_size(self._c()))

    @property
    def crc_cur(self):
        return int(self._lib.cioa_chunk_crc_cur(self._c()))

    @crc_cur.setter
    def crc_cur(self, v):
        self._lib.cioa_chunk_set_crc_cur(self._c(), v & 0xFFFFFFFF)

    @property
    def map(self):
        """The chunk's mapping as a ctypes byte array (None when down)."""
        size = ctypes.c_size_t(0)
        p = self._lib.cioa_chunk_map(self._c(), ctypes.byref(size))
        if not p:
            return None
        return (ctypes.c_char * size.value).from_address(p)

    @property
    def alloc_size(self):
        m = self.map
        return 0 if m is None else len(m)

    def hash(self):
        m = self.map
        return None if m is None else bytes(m[2:6])

    def content(self):
        m = self.map
        off = HDR_MIN + self.meta_len()
        return bytes(m[off:off + self.data_size])

    def close(self, delete=False):
        if self._h:
            self._lib.cioa_chunk_close(self._h, 1 if delete else 0)
            self._h = None


def up_batch(chunks, force=False):
    """cioa_chunk_up_batch / _up_force_batch: bring the chunks up with the
    outcome of chunk.up() / up_force() called on each in order, the verifies
    batched.  Returns the per-chunk statuses (list of int)."""
    if not chunks:
        return []
    lib = chunks[0]._lib
    n = len(chunks)
    arr = (ctypes.c_void_p * n)(*[c._c() for c in chunks])
    st = (ctypes.c_int * n)()
    fn = lib.cioa_chunk_up_force_batch if force else lib.cioa_chunk_up_batch
    fn(arr, n, st)
    return list(st)


def sync_batch(chunks):
    """cioa_chunk_sync_batch: every chunk's deferred CRC in ONE GPU pass."""
    chunks = [c for c in chunks if c is not None]
    if not chunks:
        return CIO_OK
    lib = _bind()
    arr = (ctypes.c_void_p * len(chunks))(*[c._c() for c in chunks])
    return int(lib.cioa_chunk_sync_batch(arr, len(chunks)))


class SyncJob:
    """A begun batch sync (cioa_chunk_sync_batch_begin); end() returns what
    sync_batch would have.  Ended on garbage collection if never ended."""

    def __init__(self, lib, handle):
        self._lib, self._h = lib, handle

    def end(self):
        if not self._h:
            raise ValueError("SyncJob already ended")
        h, self._h = self._h, None
        return int(self._lib.cioa_chunk_sync_batch_end(h))

    def __del__(self):
        if getattr(self, "_h", None):
            self.end()


def sync_batch_begin(chunks):
    """cioa_chunk_sync_batch_begin: the batch's CRC pass starts on a thread of
    its own; SyncJob.end() waits for it and writes the headers.  Writing,
    syncing, a transaction, down or close of one of the chunks ends the batch
    first."""
    chunks = [c for c in chunks if c is not None]
    lib = _bind()
    arr = (ctypes.c_void_p * max(1, len(chunks)))(*[c._c() for c in chunks])
    job = ctypes.c_void_p()
    if lib.cioa_chunk_sync_batch_begin(arr, len(chunks), ctypes.byref(job)) != CIO_OK:
        raise MemoryError("cioa_chunk_sync_batch_begin")
    return SyncJob(lib, job.value)


class ChunkFile(Chunk):
    """One chunk addressed by its path (root/stream/name), in a private context."""

    @classmethod
    def open(cls, path, flags=CIO_OPEN | CIO_CHECKSUM, deferred_crc=False, ctx_flags=0):
        path = os.path.abspath(path)
        stream_dir = os.path.dirname(path)
        root, stream, name = os.path.dirname(stream_dir), os.path.basename(stream_dir), os.path.basename(path)
        cflags = (flags & (CIO_CHECKSUM | CIO_FULL_SYNC | CIO_TRIM_FILES)) | ctx_flags
        if deferred_crc:
            cflags |= CIOA_DEFERRED_CRC
        ctx = Context(root, cflags | (flags & (CIO_OPEN | CIO_OPEN_RD)))
        st = ctx.stream(stream)
        c, err = st.open(name, (flags & (CIO_OPEN | CIO_OPEN_RD)) or CIO_OPEN)
        if c is None:
            cf = cls.__new__(cls)
            cf.ctx, cf._h, cf._lib, cf.path = ctx, None, ctx._lib, path
            cf._open_error = ctx.last_chunk_error
            return cf, err
        cf = cls(ctx, c._h)
        ctx._chunks[-1] = cf
        cf.path = path
        return cf, CIO_OK

    @property
    def error(self):
        if not self._h:
            return getattr(self, "_open_error", 0)
        return super().error

    def close(self, delete=False):
        super().close(delete)
        self.ctx.close()


def perf_write(root, data, files=1000, writes=5, batch=100, flags=CIO_CHECKSUM | CIOA_DEFERRED_CRC):
    """BASELINE config 1's loop through the C layer (cioa_bench_perf_write):
    (seconds, bytes)."""
    lib = _bind()
    buf = np.frombuffer(bytes(data), np.uint8)
    secs, nb = ctypes.c_double(0), ctypes.c_uint64(0)
    rc = lib.cioa_bench_perf_write(os.fsencode(root), buf.ctypes.data, buf.size, files, writes, batch, flags,
                                   ctypes.byref(secs), ctypes.byref(nb))
    if rc != CIO_OK:
        raise _lib.CioGpuError(f"cioa_bench_perf_write failed: {_lib.lib().cio_gpu_last_error().decode()}")
    return secs.value, int(nb.value)


def header_crc_be(path):
    with open(path, "rb") as f:
        return struct.unpack(">I", f.read(6)[2:6])[0]
