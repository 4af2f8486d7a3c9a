"""Host-side mirror of chunkio's CRC-32 interface over libchunkio_amd.so.

Names and meaning follow the reference (fluent/chunkio):

  crc_init() / crc_update(crc, data) / crc_finalize(crc)
      deps/crc32/crc32.h:74-100, deps/crc32/crc32.c:337-390 -- raw state in
      and out; crc_update on host bytes runs the library's scalar CPU path
      (the drop-in `crc_update` symbol).
  Crc32Plan / crc32_batch_dev()
      the batched GPU path: N x cio_file_calculate_checksum()
      (src/cio_file.c:66-94) over device-resident chunk contents.
  crc32_shift() / crc32_combine()
      GF(2) helpers to fold GPU partial CRCs into a running crc_cur
      (src/cio_file.c:97-113).

torch is used only as the device-memory container (tensors on cuda:N); every
CRC computation goes through the C ABI.  There is no CPU fallback for the
batched entry points: without the HIP library they raise.
"""
import ctypes

import numpy as np

from . import _lib

CRC_INIT = 0xFFFFFFFF


def crc_init():
    return CRC_INIT


def crc_finalize(crc):
    return (crc ^ 0xFFFFFFFF) & 0xFFFFFFFF


def _as_bytes(data):
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data).view(np.uint8)
    return np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)


def crc_update(crc, data):
    """crc_update(crc, data, len) of the reference on host memory."""
    buf = _as_bytes(data)
    ptr = buf.ctypes.data if buf.size else None
    return int(_lib.lib().crc_update(crc & 0xFFFFFFFFFFFFFFFF, ptr, buf.size))


def crc32(data, seed=CRC_INIT):
    """Finalized CRC-32 (zlib-compatible) of host bytes."""
    return crc_finalize(crc_update(seed, data))


def crc32_shift(raw_state, nbytes):
    return int(_lib.lib().cio_crc32_shift(raw_state & 0xFFFFFFFF, nbytes))


def crc32_combine(raw_a, raw0_b, len_b):
    return int(_lib.lib().cio_crc32_combine(raw_a & 0xFFFFFFFF, raw0_b & 0xFFFFFFFF, len_b))


def _u64_array(values):
    arr = np.ascontiguousarray(np.asarray(values, dtype=np.uint64))
    return arr, arr.ctypes.data_as(_lib.c_u64_p)


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream_ptr(stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(int(stream.cuda_stream))


class Crc32Plan:
    """Geometry of one batch (chunk offsets/lengths relative to a base).

    exec() enqueues the CRC kernels on a stream with no host synchronisation.
    """

    def __init__(self, offs, lens):
        self._offs, po = _u64_array(offs)
        self._lens, pl = _u64_array(lens)
        if self._offs.shape != self._lens.shape:
            raise ValueError("offs and lens must have the same length")
        self.n = int(self._offs.size)
        handle = ctypes.c_void_p()
        _lib.check(_lib.lib().cio_crc32_plan_create(ctypes.byref(handle), po, pl, self.n),
                   "cio_crc32_plan_create")
        self._handle = handle

    @property
    def bytes(self):
        return int(_lib.lib().cio_crc32_plan_bytes(self._handle))

    @property
    def workgroups(self):
        """Workgroups one launch runs (one per CU, or four for long mixed batches)."""
        return int(_lib.lib().cio_crc32_plan_workgroups(self._handle))

    def kernel_name(self):
        """The kernel this plan launches (crc32_stream_kernel / crc32_small_kernel)."""
        return _lib.lib().cio_crc32_plan_kernel(self._handle).decode()

    def exec(self, base, out, seeds=None, stream=None):
        """base: uint8 cuda tensor; out: int32/uint32 cuda tensor of n; seeds: same or None."""
        _lib.check(_lib.lib().cio_crc32_plan_exec(self._handle, _ptr(base), _ptr(seeds), _ptr(out),
                                                  _stream_ptr(stream)),
                   "cio_crc32_plan_exec")

    def exec_events(self, base, out, ev_start, ev_stop, seeds=None, stream=None):
        """exec() with HIP events recorded around the main kernel only."""
        _lib.check(_lib.lib().cio_crc32_plan_exec_events(self._handle, _ptr(base), _ptr(seeds),
                                                         _ptr(out), _stream_ptr(stream),
                                                         ev_start, ev_stop),
                   "cio_crc32_plan_exec_events")

    def close(self):
        if getattr(self, "_handle", None):
            _lib.lib().cio_crc32_plan_destroy(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class Crc32Ring:
    """`depth` plans of one geometry on their own streams (cio_crc32_ring_*):
    exec() queues a batch behind the caller stream's earlier work without
    making that stream wait for it, so consecutive batches overlap at their
    kernel edges; join() makes the caller stream wait for every batch queued
    so far (read the outputs after it)."""

    def __init__(self, offs, lens, depth=2):
        self._offs, po = _u64_array(offs)
        self._lens, pl = _u64_array(lens)
        if self._offs.shape != self._lens.shape:
            raise ValueError("offs and lens must have the same length")
        self.n = int(self._offs.size)
        handle = ctypes.c_void_p()
        _lib.check(_lib.lib().cio_crc32_ring_create(ctypes.byref(handle), po, pl, self.n, int(depth)),
                   "cio_crc32_ring_create")
        self._handle = handle

    def exec(self, base, out, seeds=None, stream=None):
        _lib.check(_lib.lib().cio_crc32_ring_exec(self._handle, _ptr(base), _ptr(seeds), _ptr(out),
                                                  _stream_ptr(stream)),
                   "cio_crc32_ring_exec")

    def join(self, stream=None):
        _lib.check(_lib.lib().cio_crc32_ring_join(self._handle, _stream_ptr(stream)), "cio_crc32_ring_join")

    def close(self):
        if getattr(self, "_handle", None):
            _lib.lib().cio_crc32_ring_destroy(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _to_u32_numpy(t):
    return t.cpu().numpy().view(np.uint32).copy()


def crc32_batch_dev(base, offs, lens, seeds=None, stream=None):
    """Raw CRC state of every chunk of a device-resident batch (numpy uint32)."""
    import torch
    n = len(offs)
    out = torch.empty(n, dtype=torch.int32, device=base.device)
    seeds_t = None
    if seeds is not None:
        seeds_t = torch.from_numpy(np.asarray(seeds, dtype=np.uint32).view(np.int32)).to(base.device)
    offs_arr = np.ascontiguousarray(np.asarray(offs, dtype=np.uint64))
    lens_arr = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64))
    _lib.check(_lib.lib().cio_crc32_batch_dev(_ptr(base), offs_arr.ctypes.data_as(_lib.c_u64_p),
                                              lens_arr.ctypes.data_as(_lib.c_u64_p), _ptr(seeds_t),
                                              _ptr(out), n, _stream_ptr(stream)),
               "cio_crc32_batch_dev")
    return _to_u32_numpy(out)


def crc32_batch_host(bufs, seeds=None, devices=None):
    """Raw CRC states of host buffers via pinned staging + H2D + GPU kernels.
    devices: GPU ordinals to spread the batch over (chunk i -> devices[i %
    len]); None = the current device."""
    arrays = [_as_bytes(b) for b in bufs]
    n = len(arrays)
    ptrs = (ctypes.c_void_p * max(n, 1))(*[a.ctypes.data if a.size else None for a in arrays])
    lens = (ctypes.c_size_t * max(n, 1))(*[a.size for a in arrays])
    out = np.zeros(max(n, 1), dtype=np.uint32)
    seeds_p = None
    if seeds is not None:
        seeds_arr = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint32))
        seeds_p = seeds_arr.ctypes.data_as(_lib.c_u32_p)
    if devices:
        devs = (ctypes.c_int * len(devices))(*devices)
        _lib.check(_lib.lib().cio_crc32_batch_host_multi(ptrs, lens, seeds_p, out.ctypes.data_as(_lib.c_u32_p),
                                                         n, devs, len(devices)),
                   "cio_crc32_batch_host_multi")
        return out[:n]
    _lib.check(_lib.lib().cio_crc32_batch_host(ptrs, lens, seeds_p,
                                               out.ctypes.data_as(_lib.c_u32_p), n),
               "cio_crc32_batch_host")
    return out[:n]


def crc32_batch_host_packed(host, offs, lens, seeds=None, devices=None):
    """crc32_batch_host over chunks packed in ONE host array: chunk i is
    host[offs[i]:offs[i] + lens[i]].  The pointer array is built with one numpy
    add instead of a Python object per chunk (the C call is the same)."""
    host = np.ascontiguousarray(host).view(np.uint8).reshape(-1)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    n = len(lens)
    if n and int((offs + lens).max()) > host.size:
        raise ValueError("crc32_batch_host_packed: chunk past the end of the host array")
    ptrs = offs + np.uint64(host.ctypes.data)
    out = np.zeros(max(n, 1), dtype=np.uint32)
    seeds_p = None
    if seeds is not None:
        seeds_arr = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint32))
        seeds_p = seeds_arr.ctypes.data_as(_lib.c_u32_p)
    P = ctypes.POINTER
    pp = ptrs.ctypes.data_as(P(ctypes.c_void_p))
    lp = lens.ctypes.data_as(P(ctypes.c_size_t))
    op = out.ctypes.data_as(_lib.c_u32_p)
    if devices:
        devs = (ctypes.c_int * len(devices))(*devices)
        _lib.check(_lib.lib().cio_crc32_batch_host_multi(pp, lp, seeds_p, op, n, devs, len(devices)),
                   "cio_crc32_batch_host_multi")
    else:
        _lib.check(_lib.lib().cio_crc32_batch_host(pp, lp, seeds_p, op, n), "cio_crc32_batch_host")
    return out[:n]


def crc32_split_host(buf, seed=CRC_INIT, devices=None):
    """Raw crc_update(seed, buf) of ONE host buffer split over `devices`
    (cio_crc32_split_host_multi: a piece per device, joined with
    cio_crc32_combine)."""
    arr = np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
    out = ctypes.c_uint32(0)
    devs = (ctypes.c_int * len(devices))(*devices) if devices else None
    _lib.check(_lib.lib().cio_crc32_split_host_multi(arr.ctypes.data if arr.size else None, arr.size,
                                                     seed & 0xFFFFFFFF, ctypes.byref(out), devs,
                                                     len(devices) if devices else 0),
               "cio_crc32_split_host_multi")
    return int(out.value)


def crc32_batch_cpu_packed(host, offs, lens, seeds=None, threads=1):
    """The same batch as crc32_batch_host_packed on the host CPU
    (cio_crc32_batch_cpu: the library's crc_update on `threads` threads)."""
    host = np.ascontiguousarray(host).view(np.uint8).reshape(-1)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    n = len(lens)
    if n and int((offs + lens).max()) > host.size:
        raise ValueError("crc32_batch_cpu_packed: chunk past the end of the host array")
    ptrs = offs + np.uint64(host.ctypes.data)
    out = np.zeros(max(n, 1), dtype=np.uint32)
    seeds_p = None
    if seeds is not None:
        seeds_arr = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint32))
        seeds_p = seeds_arr.ctypes.data_as(_lib.c_u32_p)
    P = ctypes.POINTER
    _lib.check(_lib.lib().cio_crc32_batch_cpu(ptrs.ctypes.data_as(P(ctypes.c_void_p)),
                                              lens.ctypes.data_as(P(ctypes.c_size_t)), seeds_p,
                                              out.ctypes.data_as(_lib.c_u32_p), n, int(threads)),
               "cio_crc32_batch_cpu")
    return out[:n]


def host_threads(threads=None):
    """The chunk layer's host CRC thread count (cio_crc32_host_threads); with
    an argument, set it first (cio_crc32_set_host_threads)."""
    if threads is not None:
        _lib.lib().cio_crc32_set_host_threads(int(threads))
    return int(_lib.lib().cio_crc32_host_threads())


def route(cpu_max=None, threads=None, reset=False, split=None):
    """The chunk layer's host/GPU route (crc_route.c): reset=True drops earlier
    settings; cpu_max (bytes, -1 = every batch on the host, 0 = every batch on
    the GPU alone) and threads set the threshold and the host thread count;
    split turns the split route (a GPU-bound batch shared with the host) on or
    off.  Returns (cpu_max, threads) in effect."""
    lib = _lib.lib()
    if reset:
        lib.cio_crc32_route_reset()
    if split is not None:
        lib.cio_crc32_set_split_route(2 if split == "force" else 1 if split else 0)
    if cpu_max is not None:
        lib.cio_crc32_set_cpu_max(ctypes.c_size_t(cpu_max).value)
    if threads is not None:
        lib.cio_crc32_set_host_threads(int(threads))
    return int(lib.cio_crc32_cpu_max()), int(lib.cio_crc32_host_threads())


def split_rates(forget=False):
    """The rates (GB/s) the split route sizes its next split with
    (cio_crc32_split_rates); forget=True drops the learned ones first."""
    lib = _lib.lib()
    if forget:
        lib.cio_crc32_split_forget()
    v = (ctypes.c_double * 6)()
    lib.cio_crc32_split_rates(v, 6)
    return dict(zip(("host_mem_t1", "host_fd_t1", "host_mem_t", "host_fd_t", "gpu_mem", "gpu_fd"),
                    (round(x, 2) for x in v)))


def device_count():
    """Visible GPUs (cio_gpu_device_count)."""
    return int(_lib.lib().cio_gpu_device_count())


def pipe_last_timing():
    """Host legs of the last host/file batch (cio_gpu_pipe_last_timing), ms."""
    v = (ctypes.c_double * 6)()
    _lib.check(_lib.lib().cio_gpu_pipe_last_timing(v, 6), "cio_gpu_pipe_last_timing")
    return {"total_ms": round(v[0], 3), "copy_ms": round(v[1], 3), "slot_wait_ms": round(v[2], 3),
            "plan_ms": round(v[3], 3), "groups": int(v[4]), "staged_bytes": int(v[5])}


def plan_cache_stats():
    """The host pipelines' plan image caches (cio_gpu_plan_cache_stats),
    summed over the idle pipelines of every device."""
    v = (ctypes.c_uint64 * 7)()
    _lib.check(_lib.lib().cio_gpu_plan_cache_stats(v, 7), "cio_gpu_plan_cache_stats")
    return dict(zip(("entries", "bytes", "hits", "misses", "stores", "evictions", "pipelines"), map(int, v)))


def host_register(arr):
    """Pin a long-lived host buffer (numpy array / mmap view) in place so that
    crc32_batch_host DMAs chunks inside it directly (no staging copy)."""
    a = _as_bytes(arr)
    _lib.check(_lib.lib().cio_crc32_host_register(a.ctypes.data, a.size), "cio_crc32_host_register")


def host_unregister(arr):
    a = _as_bytes(arr)
    _lib.check(_lib.lib().cio_crc32_host_unregister(a.ctypes.data), "cio_crc32_host_unregister")


def fill_synthetic(base, offs, lens, seed, ids=None, stream=None):
    """Fill chunks of a device buffer with the deterministic splitmix64 generator
    (chunk i uses generator index ids[i], default i)."""
    offs_arr = np.ascontiguousarray(np.asarray(offs, dtype=np.uint64))
    lens_arr = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64))
    ids_p = None
    if ids is not None:
        ids_arr = np.ascontiguousarray(np.asarray(ids, dtype=np.uint64))
        assert ids_arr.shape == offs_arr.shape
        ids_p = ids_arr.ctypes.data_as(_lib.c_u64_p)
    _lib.check(_lib.lib().cio_gpu_fill_synthetic(_ptr(base), offs_arr.ctypes.data_as(_lib.c_u64_p),
                                                 lens_arr.ctypes.data_as(_lib.c_u64_p), ids_p,
                                                 len(offs_arr), seed, _stream_ptr(stream)),
               "cio_gpu_fill_synthetic")


def sha1_batch_dev(base, offs, lens, stream=None):
    """SHA-1 digests (n x 20 bytes, numpy uint8) of a device-resident batch."""
    import torch
    n = len(offs)
    out = torch.empty(max(n, 1) * 20, dtype=torch.uint8, device=base.device)
    offs_arr = np.ascontiguousarray(np.asarray(offs, dtype=np.uint64))
    lens_arr = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64))
    _lib.check(_lib.lib().cio_sha1_batch_dev(_ptr(base), offs_arr.ctypes.data_as(_lib.c_u64_p),
                                             lens_arr.ctypes.data_as(_lib.c_u64_p), _ptr(out), n,
                                             _stream_ptr(stream)),
               "cio_sha1_batch_dev")
    return out[: n * 20].cpu().numpy().reshape(n, 20)


def sha1_batch_dev_async(base, dev_offs, dev_lens, dev_digests, stream=None):
    """Launch SHA-1 over a batch whose offsets/lengths are device tensors (int64,
    n each) into dev_digests (uint8, >= 20 n); no allocation, no sync."""
    n = int(dev_offs.numel())
    assert dev_lens.numel() == n and dev_digests.numel() >= 20 * n
    _lib.check(_lib.lib().cio_sha1_batch_dev_async(_ptr(base), _ptr(dev_offs), _ptr(dev_lens), _ptr(dev_digests),
                                                   n, _stream_ptr(stream)),
               "cio_sha1_batch_dev_async")


SHA1_STATE_BYTES = 96     # sizeof(cio_sha1_state) == sizeof(OpenSSL's SHA_CTX)


class Sha1:
    """chunkio's struct cio_sha1 (include/chunkio_amd/cio_sha1.h) on the
    library's host SHA-1: cio_sha1_init / update / final (src/cio_sha1.c:
    26-39).  `state` is the 96-byte SHA_CTX, OpenSSL's layout byte for byte,
    so it can be handed to the GPU batch calls (sha1_update_batch_dev) or to
    OpenSSL, and back."""

    def __init__(self, state=None):
        self._lib = _lib.lib()
        self._ctx = ctypes.create_string_buffer(SHA1_STATE_BYTES)
        if state is None:
            self._lib.cio_sha1_init(self._ctx)
        else:
            state = bytes(state)
            if len(state) != SHA1_STATE_BYTES:
                raise ValueError(f"a SHA_CTX is {SHA1_STATE_BYTES} bytes, got {len(state)}")
            ctypes.memmove(self._ctx, state, SHA1_STATE_BYTES)

    def update(self, data):
        b = _as_bytes(data)
        self._lib.cio_sha1_update(self._ctx, b.ctypes.data, b.size)
        return self

    def final(self):
        """cio_sha1_final: the 20-byte digest; the context is finished after
        it, as OpenSSL's SHA1_Final leaves it."""
        md = ctypes.create_string_buffer(20)
        self._lib.cio_sha1_final(md, self._ctx)
        return md.raw

    @property
    def state(self):
        return self._ctx.raw


def sha1_hash(data, want_state=False):
    """cio_sha1_hash (src/cio_sha1.c:41-57): the digest, and with want_state
    the 96-byte SHA_CTX as it was before SHA1_Final."""
    b = _as_bytes(data)
    md = ctypes.create_string_buffer(20)
    st = ctypes.create_string_buffer(SHA1_STATE_BYTES) if want_state else None
    _lib.lib().cio_sha1_hash(b.ctypes.data, b.size, md, st)
    return (md.raw, st.raw) if want_state else md.raw


def sha1_to_hex(digest):
    """cio_sha1_to_hex (src/cio_sha1.c:59-68): 40 lowercase hex digits."""
    d = ctypes.create_string_buffer(bytes(digest), 20)
    out = ctypes.create_string_buffer(41)
    _lib.lib().cio_sha1_to_hex(d, out)
    return out.value.decode()


def sha1_states_init(n, device):
    """n fresh SHA-1 contexts (SHA1_Init, cio_sha1_state_init) as a uint8
    device tensor of n x 96 bytes."""
    import torch
    host = np.zeros(max(n, 1) * SHA1_STATE_BYTES, dtype=np.uint8)
    _lib.lib().cio_sha1_state_init(host.ctypes.data, n)
    return torch.from_numpy(host[: n * SHA1_STATE_BYTES].copy()).to(device)


def sha1_states_view(states):
    """Host view of device SHA-1 contexts (SHA_CTX layout): dict of numpy
    arrays h (n x 5), Nl, Nh, bits (Nh:Nl), num (n), data (n x 64 pending
    bytes, zero past num), and raw (n x 96, the context bytes)."""
    raw = states.cpu().numpy().reshape(-1, SHA1_STATE_BYTES).copy()
    nl = raw[:, 20:24].copy().view("<u4")[:, 0]
    nh = raw[:, 24:28].copy().view("<u4")[:, 0]
    return {"h": raw[:, :20].copy().view("<u4"), "Nl": nl, "Nh": nh,
            "bits": (nh.astype(np.uint64) << np.uint64(32)) | nl.astype(np.uint64),
            "data": raw[:, 28:92].copy(), "num": raw[:, 92:96].copy().view("<u4")[:, 0], "raw": raw}


def sha1_update_batch_dev(base, dev_offs, dev_lens, states, stream=None):
    """SHA1_Update of chunk i (device tensors dev_offs/dev_lens, int64) into
    context i of `states` (sha1_states_init); one launch, no sync."""
    n = int(dev_offs.numel())
    assert dev_lens.numel() == n and states.numel() >= SHA1_STATE_BYTES * n
    _lib.check(_lib.lib().cio_sha1_update_batch_dev(_ptr(base), _ptr(dev_offs), _ptr(dev_lens), _ptr(states), n,
                                                    _stream_ptr(stream)),
               "cio_sha1_update_batch_dev")


def sha1_final_batch_dev(states, n=None, stream=None):
    """SHA1_Final of every context (left unchanged): n x 20 digest bytes (numpy)."""
    import torch
    n = states.numel() // SHA1_STATE_BYTES if n is None else n
    if n < 0 or states.numel() < n * SHA1_STATE_BYTES:
        raise ValueError(f"sha1_final_batch_dev: {n} contexts but states holds "
                         f"{states.numel() // SHA1_STATE_BYTES}")
    out = torch.empty(max(n, 1) * 20, dtype=torch.uint8, device=states.device)
    _lib.check(_lib.lib().cio_sha1_final_batch_dev(_ptr(states), _ptr(out), n, _stream_ptr(stream)),
               "cio_sha1_final_batch_dev")
    return out[: n * 20].cpu().numpy().reshape(n, 20)
