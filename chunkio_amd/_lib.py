"""ctypes binding of libchunkio_amd.so (the C ABI in include/chunkio_amd/*.h).

The shared library is built in-tree by `make` (or __graft_entry__.build()) into
chunkio_amd/lib/.  There is no fallback: if the library is missing, importing
any GPU entry point raises ImportError.
"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
# CIO_AMD_LIB: alternate build of the same ABI (A/B measurements only).
LIB_PATH = os.environ.get("CIO_AMD_LIB") or os.path.join(HERE, "lib", "libchunkio_amd.so")

# Every symbol the public headers declare (checked by tests/test_abi.py).
EXPORTS = (
    # include/crc32/crc32.h
    "crc_update",
    # include/chunkio_amd/cio_crc32_gpu.h
    "cio_gpu_init", "cio_gpu_last_error", "cio_gpu_version",
    "cio_crc32_shift", "cio_crc32_combine",
    "cio_crc32_plan_create", "cio_crc32_plan_destroy", "cio_crc32_plan_exec",
    "cio_crc32_plan_exec_events", "cio_crc32_plan_bytes", "cio_crc32_plan_kernel", "cio_crc32_plan_workgroups", "cio_crc32_ring_create", "cio_crc32_ring_exec",
    "cio_crc32_ring_join", "cio_crc32_ring_destroy", "cio_crc32_batch_dev", "cio_crc32_batch_host",
    "cio_crc32_batch_host_multi", "cio_crc32_split_host_multi", "cio_crc32_batch_fd_multi", "cio_gpu_device_count", "cio_gpu_set_device", "cio_gpu_get_device", "cio_gpu_numa_node",
    "cio_gpu_pci_bus_id", "cio_gpu_plan_cache_stats",
    "cio_crc32_host_register", "cio_crc32_host_unregister", "cio_gpu_pipe_last_timing",
    "cio_crc32_cpu_max", "cio_crc32_set_cpu_max", "cio_crc32_split_route", "cio_crc32_set_split_route", "cio_crc32_split_rates", "cio_crc32_split_forget", "cio_crc32_host_threads", "cio_crc32_set_host_threads",
    "cio_crc32_route_reset",
    "cio_crc32_batch_cpu", "cio_crc32_batch_fd_cpu",
    "cio_gpu_fill_synthetic", "cio_sha1_batch_dev", "cio_sha1_batch_dev_async",
    "cio_sha1_state_init", "cio_sha1_update_batch_dev", "cio_sha1_final_batch_dev", "cio_gpu_read_stream", "cio_gpu_read_stream_grid",
    "cio_gpu_event_create", "cio_gpu_event_destroy", "cio_gpu_event_record",
    "cio_gpu_event_elapsed_ms", "cio_gpu_stream_sync",
    # include/chunkio_amd/cio_sha1.h, include/sha1/sha1.h
    "cio_sha1_init", "cio_sha1_update", "cio_sha1_final", "cio_sha1_hash", "cio_sha1_to_hex",
    "cioa_SHA1_Init", "cioa_SHA1_Update", "cioa_SHA1_Final",
    # include/chunkio_amd/cio_verify.h
    "cio_file_verify_batch", "cio_file_verify_batch_multi", "cio_verify_paths", "cio_verify_paths_multi",
    # include/chunkio_amd/cio_sync.h
    "cio_file_sync_batch", "cio_file_sync_batch_multi", "cio_file_sync_batch_begin", "cio_file_sync_batch_end",
    # include/chunkio_amd/cioa_chunk.h
    "cioa_create", "cioa_destroy", "cioa_set_max_chunks_up", "cioa_set_realloc_size_hint",
    "cioa_enable_file_trimming", "cioa_disable_file_trimming", "cioa_get_flags", "cioa_set_devices",
    "cioa_last_chunk_error", "cioa_total_chunks", "cioa_total_chunks_up",
    "cioa_stream_create", "cioa_stream_get", "cioa_stream_size_chunks_up", "cioa_stream_chunks", "cioa_scan_stream", "cioa_scan_streams", "cioa_scan_dump",
    "cioa_chunk_open", "cioa_chunk_close", "cioa_chunk_delete", "cioa_chunk_write", "cioa_chunk_write_at",
    "cioa_chunk_sync", "cioa_chunk_sync_batch", "cioa_chunk_sync_batch_begin", "cioa_chunk_sync_batch_end",
    "cioa_chunk_get_content", "cioa_chunk_get_content_copy",
    "cioa_chunk_get_content_size", "cioa_chunk_get_content_end_pos", "cioa_chunk_is_file",
    "cioa_chunk_close_stream", "cioa_chunk_get_real_size", "cioa_chunk_hash", "cioa_chunk_lock",
    "cioa_chunk_unlock", "cioa_chunk_is_locked", "cioa_chunk_tx_begin", "cioa_chunk_tx_commit",
    "cioa_chunk_tx_rollback", "cioa_chunk_is_up", "cioa_chunk_up", "cioa_chunk_up_force",
    "cioa_chunk_up_batch", "cioa_chunk_up_force_batch", "cioa_chunk_down",
    "cioa_chunk_name", "cioa_chunk_map", "cioa_error_get", "cioa_chunk_crc_cur", "cioa_chunk_set_crc_cur",
    "cioa_meta_write", "cioa_meta_read", "cioa_meta_cmp", "cioa_meta_size", "cioa_bench_perf_write",
)

_lib = None
_hip_runtime = None

c_u64_p = ctypes.POINTER(ctypes.c_uint64)
c_u32_p = ctypes.POINTER(ctypes.c_uint32)


def _bind(lib):
    V, P = ctypes.c_void_p, ctypes.POINTER
    sig = {
        "crc_update": (ctypes.c_uint64, [ctypes.c_uint64, V, ctypes.c_size_t]),
        "cio_gpu_init": (ctypes.c_int, []),
        "cio_gpu_last_error": (ctypes.c_char_p, []),
        "cio_gpu_version": (ctypes.c_char_p, []),
        "cio_crc32_shift": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint64]),
        "cio_crc32_combine": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]),
        "cio_crc32_plan_create": (ctypes.c_int, [P(V), c_u64_p, c_u64_p, ctypes.c_size_t]),
        "cio_crc32_plan_destroy": (None, [V]),
        "cio_crc32_plan_exec": (ctypes.c_int, [V, V, V, V, V]),
        "cio_crc32_plan_exec_events": (ctypes.c_int, [V, V, V, V, V, V, V]),
        "cio_crc32_plan_bytes": (ctypes.c_uint64, [V]),
        "cio_crc32_plan_kernel": (ctypes.c_char_p, [V]),
        "cio_crc32_plan_workgroups": (ctypes.c_uint32, [V]),
        "cio_crc32_ring_create": (ctypes.c_int, [ctypes.POINTER(V), ctypes.POINTER(ctypes.c_uint64),
                                                 ctypes.POINTER(ctypes.c_uint64), ctypes.c_size_t, ctypes.c_int]),
        "cio_crc32_ring_exec": (ctypes.c_int, [V, V, V, V, V]),
        "cio_crc32_ring_join": (ctypes.c_int, [V, V]),
        "cio_crc32_ring_destroy": (None, [V]),
        "cio_crc32_batch_dev": (ctypes.c_int, [V, c_u64_p, c_u64_p, V, V, ctypes.c_size_t, V]),
        "cio_crc32_batch_host": (ctypes.c_int, [P(V), P(ctypes.c_size_t), c_u32_p, c_u32_p,
                                                ctypes.c_size_t]),
        "cio_crc32_batch_host_multi": (ctypes.c_int, [P(V), P(ctypes.c_size_t), c_u32_p, c_u32_p,
                                                      ctypes.c_size_t, P(ctypes.c_int), ctypes.c_int]),
        "cio_crc32_split_host_multi": (ctypes.c_int, [V, ctypes.c_size_t, ctypes.c_uint32, c_u32_p,
                                                      P(ctypes.c_int), ctypes.c_int]),
        "cio_gpu_device_count": (ctypes.c_int, []),
        "cio_gpu_set_device": (ctypes.c_int, [ctypes.c_int]),
        "cio_gpu_get_device": (ctypes.c_int, []),
        "cio_gpu_numa_node": (ctypes.c_int, [ctypes.c_int]),
        "cio_gpu_pci_bus_id": (ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
        "cio_gpu_plan_cache_stats": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
        "cio_crc32_host_register": (ctypes.c_int, [V, ctypes.c_size_t]),
        "cio_crc32_host_unregister": (ctypes.c_int, [V]),
        "cio_gpu_pipe_last_timing": (ctypes.c_int, [P(ctypes.c_double), ctypes.c_int]),
        "cio_crc32_cpu_max": (ctypes.c_size_t, []),
        "cio_crc32_set_cpu_max": (None, [ctypes.c_size_t]),
        "cio_crc32_split_route": (ctypes.c_int, []),
        "cio_crc32_set_split_route": (None, [ctypes.c_int]),
        "cio_crc32_split_rates": (None, [ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
        "cio_crc32_split_forget": (None, []),
        "cio_crc32_host_threads": (ctypes.c_int, []),
        "cio_crc32_set_host_threads": (None, [ctypes.c_int]),
        "cio_crc32_route_reset": (None, []),
        "cio_crc32_batch_cpu": (ctypes.c_int, [P(V), P(ctypes.c_size_t), c_u32_p, c_u32_p, ctypes.c_size_t,
                                               ctypes.c_int]),
        "cio_crc32_batch_fd_cpu": (ctypes.c_int, [P(ctypes.c_int), c_u64_p, P(ctypes.c_size_t), c_u32_p, c_u32_p,
                                                  ctypes.c_size_t, ctypes.c_int]),
        "cio_gpu_fill_synthetic": (ctypes.c_int, [V, c_u64_p, c_u64_p, c_u64_p, ctypes.c_size_t,
                                                  ctypes.c_uint64, V]),
        "cio_sha1_batch_dev": (ctypes.c_int, [V, c_u64_p, c_u64_p, V, ctypes.c_size_t, V]),
        "cio_sha1_batch_dev_async": (ctypes.c_int, [V, V, V, V, ctypes.c_size_t, V]),
        "cio_sha1_state_init": (None, [V, ctypes.c_size_t]),
        "cio_sha1_update_batch_dev": (ctypes.c_int, [V, V, V, V, ctypes.c_size_t, V]),
        "cio_sha1_final_batch_dev": (ctypes.c_int, [V, V, ctypes.c_size_t, V]),
        "cio_sha1_init": (None, [V]),
        "cio_sha1_update": (None, [V, V, ctypes.c_ulong]),
        "cio_sha1_final": (None, [V, V]),
        "cio_sha1_hash": (None, [V, ctypes.c_ulong, V, V]),
        "cio_sha1_to_hex": (None, [V, V]),
        "cioa_SHA1_Init": (ctypes.c_int, [V]),
        "cioa_SHA1_Update": (ctypes.c_int, [V, V, ctypes.c_size_t]),
        "cioa_SHA1_Final": (ctypes.c_int, [V, V]),
        "cio_gpu_read_stream": (ctypes.c_int, [V, ctypes.c_uint64, V]),
        "cio_gpu_read_stream_grid": (ctypes.c_int, [V, ctypes.c_uint64, ctypes.c_uint32, V]),
        "cio_gpu_event_create": (V, []),
        "cio_gpu_event_destroy": (None, [V]),
        "cio_gpu_event_record": (ctypes.c_int, [V, V]),
        "cio_gpu_event_elapsed_ms": (ctypes.c_float, [V, V]),
        "cio_gpu_stream_sync": (ctypes.c_int, [V]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("CIO_AMD_LIB") and not hasattr(lib, name):
            continue   # an older A/B build without this entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def _elf_dynamic_strings(path):
    """(SONAME, [NEEDED...]) of a 64-bit little-endian ELF shared object, read
    from its dynamic section; (None, []) if the file cannot be parsed."""
    import struct
    try:
        with open(path, "rb") as f:
            data = f.read()
        if data[:4] != b"\x7fELF" or data[4] != 2 or data[5] != 1:
            return None, []
        shoff, = struct.unpack_from("<Q", data, 0x28)
        shentsize, shnum = struct.unpack_from("<HH", data, 0x3A)
        secs = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
        dyn = [sec for sec in secs if sec[1] == 6]           # SHT_DYNAMIC
        if not dyn:
            return None, []
        _, _, _, _, off, size, link, _, _, _ = dyn[0]
        stroff = secs[link][4]

        def cstr(o):
            return data[stroff + o:data.index(b"\0", stroff + o)].decode()
        soname, needed = None, []
        for k in range(size // 16):
            tag, val = struct.unpack_from("<qQ", data, off + 16 * k)
            if tag == 0:
                break
            if tag == 1:
                needed.append(cstr(val))
            elif tag == 14:
                soname = cstr(val)
        return soname, needed
    except (OSError, ValueError, IndexError, struct.error):
        return None, []


def _pin_hip_runtime():
    """Make the library share ONE HIP runtime with torch in this process.

    libchunkio_amd.so needs libamdhip64.so.7 (RUNPATH /opt/rocm).  torch ships
    its own copy under torch/lib and loads it by path, so if this library is
    loaded before torch the process ends up with two HIP/HSA runtimes; whichever
    initialises second sees no device ("hipGetDevice: no ROCm-capable device").
    Loading torch's copy first (RTLD_GLOBAL, without importing torch) lets the
    soname match it, and torch's later import reuses the same file.
    CIOA_HIP_RUNTIME=system keeps the /opt/rocm runtime; a path picks that file.
    """
    choice = os.environ.get("CIOA_HIP_RUNTIME", "")
    if choice == "system" or "torch" in sys.modules:
        return None                 # torch already loaded: the soname matches its copy
    path = choice
    if not path:
        import importlib.util
        spec = importlib.util.find_spec("torch")
        if spec is None or not spec.origin:
            return None
        path = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
        if not os.path.exists(path):
            return None
        # Pin torch's copy only if it IS the runtime this library links: same
        # SONAME as the library's libamdhip64 DT_NEEDED entry.  A torch built
        # against another major version would otherwise add a second runtime
        # (and one this library never uses).
        soname, _ = _elf_dynamic_strings(path)
        _, needed = _elf_dynamic_strings(LIB_PATH)
        want = [x for x in needed if x.startswith("libamdhip64")]
        if soname is None or not want or soname not in want:
            import warnings
            warnings.warn(f"chunkio_amd: not pinning {path} (SONAME {soname}) for {LIB_PATH} "
                          f"(needs {want or 'no libamdhip64'}); load torch first if both are used")
            return None
    return ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


def lib():
    """Load (once) and return the bound library; raise ImportError if absent."""
    global _lib, _hip_runtime
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is not built: run `make` or __graft_entry__.build()")
        _hip_runtime = _pin_hip_runtime()   # kept referenced for the process's lifetime
        _lib = _bind(ctypes.CDLL(LIB_PATH))
    return _lib


class CioGpuError(RuntimeError):
    pass


def check(rc, what):
    if rc != 0:
        msg = lib().cio_gpu_last_error()
        raise CioGpuError(f"{what} failed: {msg.decode() if msg else 'unknown error'}")
