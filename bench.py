#!/usr/bin/env python3
"""Benchmark: device-resident batched CRC-32 on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg3|cfg4|cfg4k|sha1|e2e|perf|verify]

One "step" = one pass of the hot path over one batch: crc_update(init, chunk)
for every chunk of the batch (main kernel + per-chunk fold), inputs already
resident in HBM.  Default workload = BASELINE config 2: 1024 x 409,600-byte
chunks per GPU (weak scaling: chunk i of the N*1024-chunk job lives on GPU
i mod N; no collective on the data path).  Batches rotate over 4 device
buffers (1.68 GB) so the 256 MiB Infinity Cache cannot serve repeats.

Prints ONE JSON line (rank 0).  `value` = bytes of all ranks x K / wall time
of the K timed launches (max over ranks).  `roofline.achieved` = algorithmic
bytes per launch of the CRC kernel (sum of chunk lengths) / its average launch
duration: one HIP event pair recorded on the launch stream around the K
back-to-back timed launches, divided by K.  That average includes the short
GPU-side gaps between back-to-back kernels, but it is NOT an upper bound on
rocprofv3 --kernel-trace's per-dispatch mean: under the profiler every
dispatch carries its own completion signal and runs ~0.3-2 % longer, so the
two agree to within ~2 % either way (profiles/r03/README.md pairs them run
by run).  Launches bracketed
one by one with their own events (perturbed: the event packets serialise the
queue) are reported after the timed region as `isolated_launch_ms`.  `roofline.read_stream` is the
same-box ceiling for the access pattern: a read-only kernel with the CRC
kernel's grid and loads over the same rotating buffers (no CRC).
`cpu_baseline` (rank 0, N=1) times the reference's own deps/crc32/crc32.c
(oracle/_ref, single thread) over the same batch and checks the GPU CRCs
against it bit for bit.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
try:
    # the process's CPUs before any leg binds it to its GPU's NUMA node
    # (bind_to_gpu_node); the all-devices leg runs on all of them again
    ORIG_AFFINITY = os.sched_getaffinity(0)
except AttributeError:
    ORIG_AFFINITY = None
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
N_ROTATE = 4
METRIC = "device-resident CRC32 GB/s over N×400KB chunks; % HBM-read roofline"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=500)
    p.add_argument("--warmup", type=int, default=200)
    p.add_argument("--config", default="cfg2",
                   choices=["cfg2", "cfg3", "cfg4", "cfg4k", "sha1", "e2e", "perf", "verify", "multi"])
    p.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    p.add_argument("--no-extra", action="store_true",
                   help="cfg2 only: skip the 4 KiB (cfg4k) and 4 MiB (cfg4) lines reported in 'other_chunk_sizes'")
    p.add_argument("--ramp-ms", type=float, default=200.0,
                   help="untimed device ramp before the warmup steps (clocks/TLB; not counted as steps)")
    return p.parse_args()


def pg_timeout_s():
    """Bound on every gloo rendezvous, barrier and scalar reduction: a rank that
    dies leaves the others blocked for at most this long (gloo's default is 30
    minutes).  The longest legitimate wait between ranks is one stage's skew
    (seconds)."""
    return float(os.environ.get("CIO_BENCH_PG_TIMEOUT_S", "300"))


def init_gloo_quiet():
    """init_process_group("gloo") from the launcher's env, with a bounded
    timeout.  gloo's C++ side prints "[Gloo] Rank r is connected ..." on fd 1
    while the mesh connects; fd 1 goes to stderr meanwhile, so rank 0's stdout
    holds the JSON line alone."""
    import datetime
    import torch.distributed as dist
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=pg_timeout_s()))
        dist.barrier()
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    return dist


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Test hook (tests/test_distributed.py): CIO_BENCH_FAIL_RANK=r makes rank r
    # exit 1 before the rendezvous (CIO_BENCH_FAIL_AT=init), after it while
    # the others wait in a barrier as they would in the timed region
    # (=barrier, the default), or hang there (=hang).  The launcher must end
    # the job promptly in every case, not wait for gloo's timeout.
    fail_rank = os.environ.get("CIO_BENCH_FAIL_RANK")
    fail_at = os.environ.get("CIO_BENCH_FAIL_AT", "barrier")
    failing = fail_rank is not None and int(fail_rank) == rank
    if failing and fail_at == "init":
        os._exit(1)
    dist = None
    if world > 1:
        # The data path has no collective (chunks shard round-robin), so no
        # RCCL communicator is created at all: the contract's barrier and the
        # two scalar reductions (max-over-ranks, per-GPU gather) run on gloo
        # over CPU tensors, for every N.  Joined before any GPU work, so a
        # rank that cannot start fails the job at once.
        dist = init_gloo_quiet()
    if fail_rank is not None:
        if failing and fail_at == "hang":
            while True:
                time.sleep(60)
        if failing:
            os._exit(1)
        barrier(dist)
    import torch
    # CIO_BENCH_REHEARSE=1: rehearse the N>1 path on a box with fewer GPUs
    # than ranks (ranks share devices round-robin, gloo for the barrier and
    # the max-over-ranks).  Never set by the driver's scaling runs.
    rehearse = os.environ.get("CIO_BENCH_REHEARSE") == "1"
    # CIO_BENCH_SHARE_DEVICES=1 (test hook): the same device sharing without
    # the rehearsal's exemption, so the topology check must fail the line.
    if rehearse or os.environ.get("CIO_BENCH_SHARE_DEVICES") == "1":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if args.gpus != world:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    return rank, world, torch.device("cuda", local), dist


def barrier(dist):
    if dist is not None:
        dist.barrier()


def max_over_ranks(x, dist, device):
    """MAX of a host scalar over ranks (gloo, CPU tensor)."""
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_over_ranks(x, dist, device):
    """[x of rank 0, x of rank 1, ...] (every rank gets the list; gloo, CPU)."""
    if dist is None:
        return [x]
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    out = [torch.zeros(1, dtype=torch.float64) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(v.item()) for v in out]


def local_topology(device):
    """Which physical GPU this rank drives: HIP device index, PCI bus ID
    (cio_gpu_pci_bus_id), NUMA node of its PCIe link, UUID, host."""
    import ctypes
    import socket
    import torch
    import chunkio_amd as cio
    idx = device.index if device.index is not None else torch.cuda.current_device()
    buf = ctypes.create_string_buffer(64)
    bus = buf.value.decode() if cio.lib().cio_gpu_pci_bus_id(idx, buf, 64) == 0 else None
    try:
        uuid = str(torch.cuda.get_device_properties(idx).uuid)
    except (AttributeError, RuntimeError):
        uuid = None
    return {"device_index": int(idx), "pci_bus_id": bus, "numa_node": int(cio.lib().cio_gpu_numa_node(idx)),
            "uuid": uuid, "host": socket.gethostname(), "pid": os.getpid()}


def gather_topology(local, dist, rehearse):
    """Every rank's local_topology() in rank order (gloo all_gather_object).
    Outside a rehearsal (CIO_BENCH_REHEARSE=1: ranks share the devices of a
    smaller box on purpose) two ranks on one (host, PCI bus ID) are a broken
    process layout: a scaling line from it would count one GPU's work N
    times, so this raises SystemExit on every rank (the launcher then fails
    the job with a non-zero status)."""
    if dist is None:
        topo = [local]
    else:
        topo = [None] * dist.get_world_size()
        dist.all_gather_object(topo, local)
    keys = [(t.get("host"), t.get("pci_bus_id")) for t in topo]
    dup = sorted({k for k in keys if keys.count(k) > 1})
    out = {"ranks": len(topo), "distinct_gpus": len(set(keys)), "rehearsal": bool(rehearse),
           "device_index": [t.get("device_index") for t in topo],
           "pci_bus_id": [t.get("pci_bus_id") for t in topo],
           "numa_node": [t.get("numa_node") for t in topo],
           "host": sorted({t.get("host") for t in topo})}
    if dup and not rehearse:
        raise SystemExit(f"bench.py: ranks share a GPU (host, PCI bus ID) {dup}: "
                         f"{[(i, k) for i, k in enumerate(keys)]}; refusing to report a {len(topo)}-GPU line")
    return out


def job_digest_matches(local, n_total, want_sha256, dist):
    """A job checked whole at any N: every rank's results (its round-robin
    shard, in shard order: raw u32 CRCs, or (n, 20) uint8 SHA-1 digests) are
    gathered to rank 0 in job order -- 4 bytes per word over gloo, after the
    timed region, not on the data path -- and the SHA-256 of the job's bytes
    (u32 little-endian / digests concatenated) compared with `want_sha256`.
    True/False on rank 0, None on the others."""
    import hashlib
    local = np.ascontiguousarray(local)
    words = local.astype(np.uint32)[:, None] if local.ndim == 1 else local.view("<u4")
    if dist is None:
        job = words
    else:
        from chunkio_amd import shard
        cols = [shard.gather_results(words[:, k], n_total, dst=0) for k in range(words.shape[1])]
        if cols[0] is None:
            return None
        job = np.stack(cols, axis=1)
    if len(job) != n_total:
        return False
    return hashlib.sha256(job.astype("<u4").tobytes()).hexdigest() == want_sha256


def weak_job_golden(cfg, world):
    """SHA-256 of the weak-scaled `cfg` job at `world` GPUs, or None if the
    fixture has none (tests/golden/make_golden.py weak_jobs: N = 1..8)."""
    with open(os.path.join(ROOT, "tests", "golden", "crc32_vectors.json")) as f:
        return json.load(f).get("weak_jobs", {}).get(cfg, {}).get(str(world))


def geometry(cfg, rank, world):
    """(lens, ids, seed, workload description, scaling) of this rank's shard."""
    from chunkio_amd import workloads as wl
    if cfg in ("cfg2", "sha1", "e2e"):
        ids = np.arange(rank, wl.CFG2_N * world, world, dtype=np.uint64)   # weak: 1024 per GPU
        lens = np.full(len(ids), wl.CFG2_LEN, dtype=np.uint64)
        desc = {"workload": "cfg2: 1024 x 409600 B chunks per GPU, device-resident, batched CRC32",
                "chunks_per_gpu": int(len(ids)), "chunk_bytes": wl.CFG2_LEN}
        return lens, ids, wl.CFG2_SEED, desc, "weak"
    if cfg == "cfg3":
        ids = np.arange(rank, wl.CFG3_N * world, world, dtype=np.uint64)  # weak: 65536 per GPU
        lens = wl.cfg3_lens(wl.CFG3_N * world)[ids.astype(np.int64)]
        rnd = int(os.environ.get("CIO_BENCH_CFG3_ROUND", "0"))
        if rnd:
            # diagnostic (traffic attribution, profiles/r05/cfg3_traffic/): every
            # length rounded up to a multiple of `rnd` (and offsets aligned to
            # it in run_crc), same kernel and grid; checks no longer apply
            lens = (lens + np.uint64(rnd - 1)) // np.uint64(rnd) * np.uint64(rnd)
        desc = {"workload": "cfg3: 65536 mixed chunks per GPU, len=floor(4096*1024^u), "
                            "persistent load-balanced kernel", "chunks_per_gpu": int(len(ids)),
                "bytes_per_gpu": int(lens.sum())}
        return lens, ids, wl.CFG3_SEED, desc, "weak"
    if cfg == "cfg4k":
        ids = np.arange(rank, wl.CFG4K_N * world, world, dtype=np.uint64)  # weak: 102400 per GPU
        lens = np.full(len(ids), wl.CFG4K_LEN, dtype=np.uint64)
        desc = {"workload": "cfg4k: 102400 x 4096 B chunks per GPU (cfg2's bytes in 4 KiB records), "
                            "small-chunk kernel", "chunks_per_gpu": int(len(ids)), "chunk_bytes": wl.CFG4K_LEN}
        return lens, ids, wl.CFG4K_SEED, desc, "weak"
    if cfg == "cfg4":
        ids = wl.shard_round_robin(wl.CFG4_N, rank, world).astype(np.uint64)  # strong: 8192 total
        lens = np.full(len(ids), wl.CFG4_LEN, dtype=np.uint64)
        desc = {"workload": "cfg4: 8192 x 4 MiB chunks per job, round-robin over GPUs",
                "chunks_total": wl.CFG4_N, "chunks_this_gpu": int(len(ids)), "chunk_bytes": wl.CFG4_LEN}
        return lens, ids, wl.CFG4_SEED, desc, "strong"
    raise ValueError(cfg)


def load_pmc_traffic(cfg, bytes_per_launch):
    """HBM bytes per launch of the main kernel, from a committed rocprofv3 --pmc
    pass: the pass's measured traffic when it profiled launches of this size,
    else its traffic/algorithmic ratio applied to this launch's bytes (a strong-
    scaled shard at N > 1 launches fewer bytes than the N = 1 pass did)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{cfg}.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("algorithmic_bytes_per_launch") == bytes_per_launch:
            return d.get("hbm_bytes_per_launch")
        return int(round(d["traffic_over_algorithmic"] * bytes_per_launch))
    except Exception:
        return None


def cpu_info():
    """The box's CPU model, nproc and this process's CPU share."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count()
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": share,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_share(world=1):
    """Host threads per GPU for the multi-thread CPU figures: the box's CPU
    share per GPU (16 on the MI355X pool, OMP_NUM_THREADS there), at most this
    process's affinity divided over the N ranks of the node."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    per_gpu = int(os.environ.get("OMP_NUM_THREADS") or 16)
    return max(1, min(per_gpu, 16, aff // max(1, world)))


def cpu_baseline(host_buf, offs, lens, gpu_out, world=1, reps=64, perf=True):
    """Reference crc_update (oracle/_ref, 1 thread) over the same batch (at
    N > 1: rank 0's shard, the same per-GPU batch size)."""
    import ctypes
    from oracle import pyoracle as po
    lib = po.ref()
    kind, prefix = "reference", "ref_"
    if lib is None:
        lib, kind, prefix = po.oracle(), "port", "oracle_"
    n = len(offs)
    out = np.zeros(n, dtype=np.uint32)
    offs_c = np.ascontiguousarray(offs, dtype=np.uint64)
    lens_c = np.ascontiguousarray(lens, dtype=np.uint64)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    # reps = 64: ~10 s of single-thread CPU work at ~2.6 GB/s (the bounded sample)
    secs = getattr(lib, prefix + "crc_batch_time")(
        host_buf.ctypes.data, offs_c.ctypes.data_as(u64p), lens_c.ctypes.data_as(u64p), n, reps,
        out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    nbytes = float(lens_c.sum()) * reps
    res = {"value": round(nbytes / secs / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": kind,
           "sample": f"{n} chunks x {int(lens_c[0]) if n else 0} B (the full per-GPU cfg2 batch) x {reps} "
                     f"passes, crc_update(init, chunk) per chunk, deps/crc32/crc32.c "
                     f"{'compiled from the reference' if kind == 'reference' else 'oracle port'}, -O3",
           "bit_exact_vs_gpu": bool(np.array_equal(out, gpu_out)), **cpu_info()}
    # the same batch over the box's CPU share (16 threads per
    # GPU there), informational; `value`/`cores` above stay the 1-thread
    # reference (chunkio itself is single-threaded).
    nt = cpu_share(world)
    f_mt = getattr(lib, prefix + "crc_batch_time_mt", None)
    if f_mt is not None:
        f_mt.restype = ctypes.c_double
        f_mt.argtypes = [ctypes.c_void_p, u64p, u64p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                         ctypes.POINTER(ctypes.c_uint32)]
        out_mt = np.zeros(n, dtype=np.uint32)
        mreps = 2 * reps
        secs_mt = f_mt(host_buf.ctypes.data, offs_c.ctypes.data_as(u64p), lens_c.ctypes.data_as(u64p), n,
                       mreps, nt, out_mt.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
        res["multi_thread"] = {"value": round(float(lens_c.sum()) * mreps / secs_mt / 1e9, 3), "unit": "GB/s",
                               "threads": nt, "bit_exact_vs_gpu": bool(np.array_equal(out_mt, gpu_out)),
                               "sample": f"same batch x {mreps} passes, chunk i on thread i % {nt}",
                               "threads_rule": f"per-GPU CPU share at N={world}: min(16, OMP_NUM_THREADS, "
                                               f"affinity_cpus // N)"}
    # The library's own host path over the same batch (crc_update with
    # VPCLMULQDQ folding, cio_crc32_batch_cpu), 1 thread and the per-GPU CPU
    # share: what a host-resident batch costs without the GPU.  Not the
    # baseline (that is the reference's crc32.c above), reported beside it.
    try:
        import chunkio_amd as cio
        lib_host = {}
        for t in sorted({1, cpu_share(world)}):
            cio.crc32_batch_cpu_packed(host_buf, offs_c, lens_c, threads=t)
            hreps = 8 if t == 1 else 32
            t0 = time.perf_counter()
            for _ in range(hreps):
                got = cio.crc32_batch_cpu_packed(host_buf, offs_c, lens_c, threads=t)
            dt = time.perf_counter() - t0
            lib_host[f"threads_{t}"] = {"GBps": round(float(lens_c.sum()) * hreps / dt / 1e9, 2),
                                        "bit_exact_vs_gpu": bool(np.array_equal(got, gpu_out))}
        lib_host["sample"] = "same batch, cio_crc32_batch_cpu (the library's host crc_update), back-to-back passes"
        res["library_host_path"] = lib_host
    except Exception as e:  # informational
        res["library_host_path"] = {"error": str(e)}
    # tools/cio -k -p restatement (BASELINE config 1), bounded sample of files.
    if not perf:
        return res
    try:
        d400 = np.fromfile(os.path.join(ROOT, "tests", "golden", "400kb.txt"), dtype=np.uint8)
        files, writes = 1000, 5
        perf = {}
        for ck in (1, 0):
            with tempfile.TemporaryDirectory(prefix="cioa-perf-") as tmp:
                nb = ctypes.c_uint64(0)
                t = getattr(lib, prefix + "cio_perf_write")(tmp.encode(), d400.ctypes.data, d400.size,
                                                            files, writes, ck, ctypes.byref(nb))
                perf["crc_on" if ck else "crc_off"] = {"seconds": round(t, 4),
                                                        "bytes_per_s": round(nb.value / t, 1)}
        res["cio_perf_k_p"] = {"sample": f"{files} files x {writes} writes x 409600 B (the reference's own config 1)",
                               **perf}
    except Exception as e:  # the perf port is informational
        res["cio_perf_k_p"] = {"error": str(e)}
    return res


def cpu_sample_baseline(dev_buf, offs, lens, gpu_out, max_bytes=1 << 30, world=1):
    """SURVEY §8(d) CPU item 2 for the cfg3 / cfg4 batches: the reference's
    crc_update (oracle/_ref) on 1 thread and on the box's per-GPU CPU share,
    over a bounded sample of the same batch (its first chunks, <= 1 GiB,
    copied from HBM), each result checked against the GPU's."""
    import ctypes
    from oracle import pyoracle as po
    lib = po.ref()
    kind, prefix = "reference", "ref_"
    if lib is None:
        lib, kind, prefix = po.oracle(), "port", "oracle_"
    k = int(max(1, np.searchsorted(np.cumsum(lens.astype(np.uint64)), max_bytes, side="right")))
    k = min(k, len(lens))
    lo, hi = int(offs[0]), int(offs[k - 1] + lens[k - 1])
    host = dev_buf[lo:hi].cpu().numpy()
    o = np.ascontiguousarray(offs[:k] - offs[0], dtype=np.uint64)
    ln = np.ascontiguousarray(lens[:k], dtype=np.uint64)
    u64p, u32p = ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32)
    out = np.zeros(k, dtype=np.uint32)
    secs = getattr(lib, prefix + "crc_batch_time")(host.ctypes.data, o.ctypes.data_as(u64p), ln.ctypes.data_as(u64p),
                                                     k, 1, out.ctypes.data_as(u32p))
    res = {"value": round(float(ln.sum()) / secs / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": kind,
           "sample": f"the batch's first {k} chunks ({int(ln.sum())} B, copied from HBM), one pass, "
                     f"crc_update(init, chunk) per chunk",
           "bit_exact_vs_gpu": bool(np.array_equal(out, gpu_out[:k]))}
    f_mt = getattr(lib, prefix + "crc_batch_time_mt", None)
    if f_mt is not None:
        f_mt.restype = ctypes.c_double
        f_mt.argtypes = [ctypes.c_void_p, u64p, u64p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, u32p]
        nt = cpu_share(world)
        out_mt = np.zeros(k, dtype=np.uint32)
        secs_mt = f_mt(host.ctypes.data, o.ctypes.data_as(u64p), ln.ctypes.data_as(u64p), k, 2, nt,
                       out_mt.ctypes.data_as(u32p))
        res["multi_thread"] = {"value": round(float(ln.sum()) * 2 / secs_mt / 1e9, 3), "unit": "GB/s", "threads": nt,
                               "bit_exact_vs_gpu": bool(np.array_equal(out_mt, gpu_out[:k]))}
    return res


def run_crc(args, rank, world, device, dist):
    import torch
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl

    lens, ids, seed, desc, scaling = geometry(args.config, rank, world)
    align = 16
    if args.config == "cfg3" and os.environ.get("CIO_BENCH_CFG3_ROUND"):
        align = max(16, int(os.environ["CIO_BENCH_CFG3_ROUND"]))
        desc["diagnostic_round"] = align
    offs = wl.packed_offsets(lens, align=align)
    total = wl.batch_bytes(offs, lens)
    nrot = N_ROTATE if total * N_ROTATE < 64e9 else 1
    bufs = []
    for b in range(nrot):
        t = torch.empty(total + 64, dtype=torch.uint8, device=device)
        cio.fill_synthetic(t, offs, lens, seed + b, ids=ids)
        bufs.append(t)
    outs = [torch.empty(len(lens), dtype=torch.int32, device=device) for _ in range(nrot)]
    plan = cio.Crc32Plan(offs, lens)
    stream = torch.cuda.current_stream(device)
    lib = cio.lib()
    sptr = int(stream.cuda_stream)

    # Device ramp (not a step): the GPU's clocks and TLBs settle over the first
    # ~100 ms of work, so short --warmup values would otherwise time a cold
    # device.  Launches of the same kernel over the same buffers, untimed.
    ramp_t0 = time.perf_counter()
    ramp_n = 0
    while time.perf_counter() - ramp_t0 < args.ramp_ms * 1e-3:
        for i in range(16):
            plan.exec(bufs[i % nrot], outs[i % nrot], stream=stream)
        torch.cuda.synchronize(device)
        ramp_n += 16
    for i in range(args.warmup):
        plan.exec(bufs[i % nrot], outs[i % nrot], stream=stream)
    torch.cuda.synchronize(device)

    # Timed region: K back-to-back launches of the single CRC kernel over the
    # rotating batches, bracketed by one HIP event pair on the launch stream
    # (average launch duration, launch gaps included) and the host clock.
    ev0, ev1 = lib.cio_gpu_event_create(), lib.cio_gpu_event_create()
    barrier(dist)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    lib.cio_gpu_event_record(ev0, sptr)
    for i in range(args.steps):
        b = i % nrot
        plan.exec(bufs[b], outs[b], stream=stream)
    lib.cio_gpu_event_record(ev1, sptr)
    torch.cuda.synchronize(device)
    barrier(dist)
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed, dist, device)
    kernel_ms = lib.cio_gpu_event_elapsed_ms(ev0, ev1) / args.steps
    outs_ref = [o.cpu().numpy().copy() for o in outs]
    lib.cio_gpu_event_destroy(ev0)
    lib.cio_gpu_event_destroy(ev1)

    # Diagnostic (after the timed region): launches each bracketed by their
    # own event pair -- the per-launch distribution, isolated launches.
    nd = min(args.steps, 100)
    evs = [(lib.cio_gpu_event_create(), lib.cio_gpu_event_create()) for _ in range(nd)]
    for i in range(nd):
        plan.exec_events(bufs[i % nrot], outs[i % nrot], evs[i][0], evs[i][1], stream=stream)
    torch.cuda.synchronize(device)
    launch_ms = np.array([lib.cio_gpu_event_elapsed_ms(a, b) for a, b in evs])
    for a, b in evs:
        lib.cio_gpu_event_destroy(a)
        lib.cio_gpu_event_destroy(b)

    # Same-box ceiling for this access pattern (read-only, no CRC), same
    # buffers, timed the same way (back-to-back under one event pair).
    wgs = plan.workgroups     # the plan's grid (one or four workgroups per CU)
    for i in range(8):
        lib.cio_gpu_read_stream_grid(bufs[i % nrot].data_ptr(), total, wgs, sptr)
    nrs = 50 if total < 4e9 else 4
    r0, r1 = lib.cio_gpu_event_create(), lib.cio_gpu_event_create()
    lib.cio_gpu_event_record(r0, sptr)
    for i in range(nrs):
        lib.cio_gpu_read_stream_grid(bufs[i % nrot].data_ptr(), total, wgs, sptr)
    lib.cio_gpu_event_record(r1, sptr)
    rs_ms = lib.cio_gpu_event_elapsed_ms(r0, r1) / nrs
    lib.cio_gpu_event_destroy(r0)
    lib.cio_gpu_event_destroy(r1)
    rs_gbs = (total // 4096 * 4096) / (rs_ms * 1e-3) / 1e9

    # Deployment figure, not the headline: consecutive batches queued on a
    # ring of two plans with their own streams (cio_crc32_ring_*), joined on
    # the launch stream after the K batches, so one batch's launch tail
    # overlaps the next batch's start, as in a service that keeps two verify
    # batches in flight.  Same K, same buffers.
    pipelined = None
    if args.config == "cfg2" and not args.no_extra:
        ring = cio.Crc32Ring(offs, lens, depth=2)
        for i in range(max(200, args.warmup)):
            ring.exec(bufs[i % nrot], outs[i % nrot], stream=stream)
        ring.join(stream=stream)
        torch.cuda.synchronize(device)
        q0, q1 = lib.cio_gpu_event_create(), lib.cio_gpu_event_create()
        lib.cio_gpu_event_record(q0, sptr)
        for i in range(args.steps):
            ring.exec(bufs[i % nrot], outs[i % nrot], stream=stream)
        ring.join(stream=stream)
        lib.cio_gpu_event_record(q1, sptr)
        torch.cuda.synchronize(device)
        pipe_ms = lib.cio_gpu_event_elapsed_ms(q0, q1) / args.steps
        for e_ in (q0, q1):
            lib.cio_gpu_event_destroy(e_)
        same = all(np.array_equal(outs[b].cpu().numpy(), outs_ref[b]) for b in range(nrot))
        ring.close()
        pipelined = {"GBps": round(int(lens.sum()) / (pipe_ms * 1e-3) / 1e9, 1), "ms_per_batch": round(pipe_ms, 5),
                     "frac_of_peak": round(int(lens.sum()) / (pipe_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "outputs_equal_sequential": bool(same),
                     "note": "K batches through cio_crc32_ring (2 plans, own streams), joined on the launch "
                             "stream: launch tails overlap the next batch; a deployment figure, not `value` "
                             "(kernel durations overlap)"}

    bytes_rank = int(lens.sum())
    # weak: every rank holds an equal shard; strong (cfg4): the whole 8192-chunk job
    bytes_all = bytes_rank * world if scaling == "weak" else int(wl.CFG4_N * wl.CFG4_LEN)
    value = bytes_all * args.steps / elapsed / 1e9
    achieved = bytes_rank / (kernel_ms * 1e-3) / 1e9

    # Correctness of the timed pass: batch 0 (seed) vs golden / CPU reference.
    plan.exec(bufs[0], outs[0], stream=stream)
    torch.cuda.synchronize(device)
    gpu0 = outs[0].cpu().numpy().view(np.uint32).copy()
    check = {}
    if args.config == "cfg2" and world == 1:
        import hashlib
        with open(os.path.join(ROOT, "tests", "golden", "crc32_vectors.json")) as f:
            g = json.load(f)["cfg2"]
        check["golden_sha256_match"] = hashlib.sha256(gpu0.astype("<u4").tobytes()).hexdigest() == \
            g["sha256_of_raw_le"]
    elif args.config == "cfg4k" and rank == 0:
        # Independent check (Python's zlib, not the oracle): every chunk.
        import zlib
        host0 = bufs[0].cpu().numpy()
        want = np.asarray([zlib.crc32(host0[int(o):int(o + n)]) ^ 0xFFFFFFFF for o, n in zip(offs, lens)],
                          dtype=np.uint32)
        check["zlib_match"] = bool(np.array_equal(want, gpu0))
    if args.config == "cfg3" and world == 1:
        # every one of the 65,536 CRCs against the reference crc32.c's digest
        import hashlib
        with open(os.path.join(ROOT, "tests", "golden", "crc32_vectors.json")) as f:
            g = json.load(f)["cfg3"]
        check["golden_sha256_match_all_chunks"] = hashlib.sha256(gpu0.astype("<u4").tobytes()).hexdigest() == \
            g["sha256_of_raw_le"]
    if args.config in ("cfg2", "cfg4k", "cfg3"):
        # The whole weak job at every N <= 8 (N x the per-GPU batch): each
        # rank's shard gathered to rank 0 in job order against the reference
        # crc32.c's digest of that job.
        want = weak_job_golden(args.config, world)
        if want is not None:
            m = job_digest_matches(gpu0, len(lens) * world, want, dist)
            if rank == 0:
                check["golden_sha256_match_full_job"] = bool(m)
    if args.config == "cfg4":
        # The whole 8192-chunk job at every N: each rank's shard gathered to
        # rank 0 in job order against the reference crc32.c's digest.
        with open(os.path.join(ROOT, "tests", "golden", "crc32_vectors.json")) as f:
            g = json.load(f)["cfg4"]
        m = job_digest_matches(gpu0, wl.CFG4_N, g["sha256_of_raw_le"], dist)
        if rank == 0:
            check["golden_sha256_match_full_job"] = bool(m)
    if args.config in ("cfg3", "cfg4"):
        # Full-size batches: 8 chunks spread over the batch (first, last and
        # evenly between), device bytes copied back and CRC'd with zlib.
        import zlib
        pick = np.unique(np.linspace(0, len(lens) - 1, 8).astype(np.int64))
        ok = True
        for i in pick:
            o, ln = int(offs[i]), int(lens[i])
            ok &= (zlib.crc32(bufs[0][o:o + ln].cpu().numpy()) ^ 0xFFFFFFFF) == int(gpu0[i])
        check["sample_zlib_match"] = bool(ok)
        check["sample_chunks"] = [int(i) for i in pick]
    if world > 1:
        # Every rank checks the first chunks of its own shard (chunk ids
        # rank, rank + N, ...; contents regenerated on the host from the chunk
        # id) against zlib; all ranks must agree.
        import zlib
        k = min(4, len(lens))
        want = [zlib.crc32(wl.gen_chunk(seed, int(ids[i]), int(lens[i]))) ^ 0xFFFFFFFF for i in range(k)]
        ok = [int(x) for x in gpu0[:k]] == want
        check["shard_sample_zlib_match_all_ranks"] = max_over_ranks(0.0 if ok else 1.0, dist, device) == 0.0

    res = {
        "metric": METRIC if args.config == "cfg2" else f"device-resident CRC32 GB/s ({args.config})",
        "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "device_ramp": {"ms": args.ramp_ms, "launches": ramp_n,
                        "note": "untimed launches before the warmup steps so short --warmup values do not "
                                "time a cold device"},
        "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64 uniform random bytes, generated in HBM)",
        "config": {**desc, "parallelism": f"replicas/shards x{world}, no collective on the data path",
                   "rotating_batches": nrot},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": load_pmc_traffic(args.config, bytes_rank),
                     "traffic_source": (f"profiles/pmc_{args.config}.json: HBM bytes per launch of this kernel "
                                        "from a committed rocprofv3 --pmc pass (FETCH_SIZE x2 gfx950 "
                                        "correction + WRITE_SIZE, separate passes; its traffic/algorithmic "
                                        "ratio when this launch's size differs); not measured in this run")
                     if load_pmc_traffic(args.config, bytes_rank) is not None else None,
                     "kernel": plan.kernel_name(), "kernel_ms_mean": round(kernel_ms, 5),
                     "timing": "HIP event pair on the launch stream around the K back-to-back timed "
                               "launches, divided by K (launch gaps included)",
                     "isolated_launch_ms": {"mean": round(float(launch_ms.mean()), 5),
                                            "median": round(float(np.median(launch_ms)), 5),
                                            "min": round(float(launch_ms.min()), 5),
                                            "note": f"{nd} launches each bracketed by its own event pair, "
                                                    "after the timed region"},
                     "algorithmic_bytes_per_launch": bytes_rank,
                     "workgroups": wgs,
                     "read_stream": {"GBps": round(rs_gbs, 1), "ms": round(rs_ms, 5), "workgroups": wgs,
                                     "note": "read-only kernel, same grid/loads/buffers, "
                                             f"{nrs} back-to-back launches under one event pair"},
                     "frac_of_read_stream": round(achieved / rs_gbs, 4)},
        "check": check,
    }
    if pipelined is not None:
        res["pipelined_two_streams"] = pipelined
    if world > 1:
        # per-GPU rates beside the aggregate `value`.
        res["per_gpu"] = {"achieved_GBps": [round(v, 1) for v in gather_over_ranks(achieved, dist, device)],
                          "kernel_ms_mean": [round(v, 5) for v in gather_over_ranks(kernel_ms, dist, device)],
                          "note": "rank order; each rank's algorithmic bytes / its kernel time"}
    # The reference CPU path beside the line at every N (rank 0, its own
    # shard: the same per-GPU batch), 1 thread plus the per-GPU CPU share.
    if rank == 0 and not args.no_cpu and args.config == "cfg2":
        host = bufs[0].cpu().numpy()
        res["cpu_baseline"] = cpu_baseline(host, offs, lens, gpu0, world=world)
    if rank == 0 and args.config in ("cfg3", "cfg4", "cfg4k") and not getattr(args, "no_cpu_sample", args.no_cpu):
        try:
            res["cpu_baseline"] = cpu_sample_baseline(bufs[0], offs, lens, gpu0, world=world)
        except Exception as e:  # informational
            res["cpu_baseline"] = {"error": str(e)}
    if "cpu_baseline" in res and world > 1:
        res["cpu_baseline"]["shard"] = f"rank 0's shard of the {world}-GPU job (the per-GPU batch)"
    plan.close()
    return res


def run_sha1(args, rank, world, device, dist):
    import hashlib
    import torch
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl
    lens, ids, seed, desc, scaling = geometry("sha1", rank, world)
    offs = wl.packed_offsets(lens, align=16)
    buf = torch.empty(wl.batch_bytes(offs, lens) + 64, dtype=torch.uint8, device=device)
    cio.fill_synthetic(buf, offs, lens, seed, ids=ids)
    # Device-resident descriptors (cio_sha1_batch_dev_async): K launches back
    # to back on the current stream, no per-call allocation or host sync.
    d_offs = torch.from_numpy(offs.astype(np.int64)).to(device)
    d_lens = torch.from_numpy(lens.astype(np.int64)).to(device)
    digests = torch.zeros(len(lens) * 20, dtype=torch.uint8, device=device)
    for _ in range(args.warmup):
        cio.sha1_batch_dev_async(buf, d_offs, d_lens, digests)
    barrier(dist)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        cio.sha1_batch_dev_async(buf, d_offs, d_lens, digests)
    torch.cuda.synchronize(device)
    barrier(dist)
    elapsed = max_over_ranks(time.perf_counter() - t0, dist, device)
    value = int(lens.sum()) * world * args.steps / elapsed / 1e9
    got = digests.cpu().numpy().reshape(-1, 20)
    sample = sorted({0, len(lens) // 2, len(lens) - 1})
    check = {"hashlib_match": all(
        bytes(got[i]) == hashlib.sha1(wl.gen_chunk(seed, int(ids[i]) if ids is not None else i,
                                                   int(lens[i])).tobytes()).digest() for i in sample),
             "sample_chunks": sample}
    want = weak_job_golden("sha1", world)
    if want is not None:
        # every digest of the N-GPU job against hashlib's, gathered to rank 0
        m = job_digest_matches(got, len(lens) * world, want, dist)
        if rank == 0:
            check["golden_sha256_match_full_job"] = bool(m)
    if world == 1:
        # all 1,024 digests against hashlib's (tests/golden/make_golden.py)
        with open(os.path.join(ROOT, "tests", "golden", "crc32_vectors.json")) as f:
            g = json.load(f)["sha1"]
        check["golden_sha256_match_all_digests"] = hashlib.sha256(got.tobytes()).hexdigest() == \
            g["cfg5_sha256_of_digests"]
    cpu = None
    if rank == 0 and not args.no_cpu:
        cpu = sha1_cpu_baseline(buf.cpu().numpy(), offs, lens, got, world)
    # The bound: one wave's issue rate on the dependent round chain
    # (tools/probe/sha1_round_probe.hip: 20.35 cycles per 5-VALU round at
    # 2.40 GHz, profiles/r02/sha1/sha1_round_probe.txt) times the longest
    # chunk's blocks (message + padding).
    max_blocks = int(((lens.astype(np.uint64) + 8) // 64 + 1).max())
    floor_s = max_blocks * 80 * 20.35 / 2.40e9
    floor_gbs = int(lens.sum()) / floor_s / 1e9
    return {"metric": "device-resident SHA-1 GB/s over N×400KB chunks (cfg5)", "value": round(value, 3),
            "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {**desc, "workload": "cfg5: SHA-1 over 1024 x 409600 B per GPU"},
            "roofline": {"bound": "valu-issue (round chain)", "achieved": round(value / world, 2),
                         "issue_floor_GBps": round(floor_gbs, 2),
                         "frac_of_issue_floor": round(value / world / floor_gbs, 4),
                         "issue_floor_source": "tools/probe/sha1_round_probe.hip: 20.35 cycles per round "
                                               "at 2.40 GHz x 80 rounds x the longest chunk's blocks",
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(value / world / HBM_PEAK_GBS, 5),
                         "traffic": load_pmc_traffic("sha1", int(lens.sum())),
                         "traffic_source": "profiles/pmc_sha1.json: HBM bytes per launch of sha1_kernel from a "
                                           "committed rocprofv3 --pmc pass; not measured in this run"
                         if load_pmc_traffic("sha1", int(lens.sum())) is not None else None},
            "timing": "K launches of cio_sha1_batch_dev_async (device-resident offsets/lengths) back to back, "
                      "host clock between stream syncs",
            "check": check, **({"cpu_baseline": cpu} if cpu is not None else {})}


def sha1_cpu_baseline(host, offs, lens, gpu_digests, world=1):
    """BASELINE.md config 5's CPU path: OpenSSL SHA-1 (Python's hashlib) over
    the same batch (rank 0's shard at N > 1), one digest per chunk as
    src/cio_sha1.c:41-57 computes it, on 1 thread and on the per-GPU CPU
    share; every digest checked against the GPU's."""
    import hashlib
    from concurrent.futures import ThreadPoolExecutor
    views = [memoryview(host[int(o):int(o) + int(n)]) for o, n in zip(offs, lens)]
    nbytes = float(np.asarray(lens, dtype=np.float64).sum())

    def digests(idx):
        return [hashlib.sha1(views[i]).digest() for i in idx]

    want = [bytes(d) for d in gpu_digests]
    t0 = time.perf_counter()
    reps = 0
    while True:                      # >= 2 s of single-thread work (the bounded sample)
        one = digests(range(len(views)))
        reps += 1
        if time.perf_counter() - t0 >= 2.0:
            break
    secs = time.perf_counter() - t0
    res = {"value": round(nbytes * reps / secs / 1e9, 4), "unit": "GB/s", "cores": 1,
           "kind": "openssl (hashlib.sha1)",
           "sample": f"{len(views)} chunks x {int(lens[0]) if len(lens) else 0} B (the whole per-GPU cfg5 batch) x "
                     f"{reps} passes, one SHA-1 per chunk",
           "bit_exact_vs_gpu": one == want,
           "note": "the reference's own SHA-1 (<sha1/sha1.h>) is not vendored; OpenSSL via hashlib is the "
                   "CPU path BASELINE.md names for config 5", **cpu_info()}
    nt = cpu_share(world)
    if nt > 1:
        parts = [list(range(t, len(views), nt)) for t in range(nt)]
        with ThreadPoolExecutor(nt) as ex:
            list(ex.map(digests, parts))                                   # warm
            mreps = 0
            t0 = time.perf_counter()
            while True:
                outs = list(ex.map(digests, parts))
                mreps += 1
                if time.perf_counter() - t0 >= 1.0:
                    break
            secs = time.perf_counter() - t0
        mt = [None] * len(views)
        for t, idx in enumerate(parts):
            for i, d in zip(idx, outs[t]):
                mt[i] = d
        res["multi_thread"] = {"value": round(nbytes * mreps / secs / 1e9, 3), "unit": "GB/s", "threads": nt,
                               "bit_exact_vs_gpu": mt == want,
                               "sample": f"same batch x {mreps} passes, chunk i on thread i % {nt} "
                                         "(hashlib releases the GIL while hashing)",
                               "threads_rule": f"per-GPU CPU share at N={world}: min(16, OMP_NUM_THREADS, "
                                               f"affinity_cpus // N)"}
    # the library's own host SHA-1 (cio_sha1_hash: the CPU's SHA extensions),
    # the host half of the SHA-1 boundary, over the same batch on 1 thread
    import chunkio_amd as cio
    cio.sha1_hash(views[0])                          # warm (library, dispatch)
    t0 = time.perf_counter()
    lreps = 0
    while True:
        lib_one = [cio.sha1_hash(v) for v in views]
        lreps += 1
        if time.perf_counter() - t0 >= 1.0:
            break
    secs = time.perf_counter() - t0
    res["library_host_path"] = {"value": round(nbytes * lreps / secs / 1e9, 4), "unit": "GB/s", "threads": 1,
                                "bit_exact_vs_gpu": lib_one == want,
                                "sample": f"same batch x {lreps} passes, cio_sha1_hash per chunk (host SHA-1 "
                                          "of include/sha1/sha1.h, SHA_CTX bytes equal OpenSSL's)"}
    if world > 1:
        res["shard"] = f"rank 0's shard of the {world}-GPU job (the per-GPU batch)"
    return res


class E2eDiag:
    """Diagnostic preambles of the e2e leg (profiles/r04/e2e_vram_free/README.md),
    all off by default: CIO_BENCH_PRE_STREAMS=k creates k HIP streams (each
    having run work) before the pipeline's own; CIO_BENCH_PRE_ALLOC_GB=g
    allocates, writes and frees g GB of HBM before the pipeline is created,
    or after its warmup calls with CIO_BENCH_ALLOC_AFTER_WARM=1, then sleeps
    CIO_BENCH_ALLOC_SETTLE_S seconds."""

    def __init__(self, device):
        self.device = device
        self.streams = []
        self.gb = float(os.environ.get("CIO_BENCH_PRE_ALLOC_GB", "0"))
        self.after = os.environ.get("CIO_BENCH_ALLOC_AFTER_WARM") == "1"

    def _alloc(self):
        import torch
        big = torch.empty(int(self.gb * 1e9), dtype=torch.uint8, device=self.device)
        big.fill_(1)
        torch.cuda.synchronize(self.device)
        del big
        torch.cuda.empty_cache()
        time.sleep(float(os.environ.get("CIO_BENCH_ALLOC_SETTLE_S", "0")))

    def before_pipeline(self):
        k = int(os.environ.get("CIO_BENCH_PRE_STREAMS", "0"))
        if k:
            import torch
            for _ in range(k):
                st = torch.cuda.Stream(self.device)
                with torch.cuda.stream(st):
                    torch.ones(16, device=self.device).sum()
                self.streams.append(st)
            torch.cuda.synchronize(self.device)
        if self.gb and not self.after:
            self._alloc()

    def after_warmup(self):
        if self.gb and self.after:
            self._alloc()


def run_e2e(args, rank, world, device, dist):
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl
    lens, ids, seed, desc, scaling = geometry("e2e", rank, world)
    bound = bind_to_gpu_node(device.index or 0)
    diag = E2eDiag(device)
    diag.before_pipeline()
    host, offs = wl.host_batch(seed, lens, align=16)
    for _ in range(max(1, args.warmup)):
        out = cio.crc32_batch_host_packed(host, offs, lens)
    diag.after_warmup()
    barrier(dist)
    t0 = time.perf_counter()
    steps = max(1, min(args.steps, 30))
    call_s = []
    for _ in range(steps):
        tc = time.perf_counter()
        out = cio.crc32_batch_host_packed(host, offs, lens)
        call_s.append(time.perf_counter() - tc)
    barrier(dist)
    elapsed = max_over_ranks(time.perf_counter() - t0, dist, device)
    value = int(lens.sum()) * world * steps / elapsed / 1e9
    legs_staged = cio.pipe_last_timing()
    # Same batch with the host buffer pinned in place once (long-lived chunk
    # mappings): the pipeline DMAs it directly, no staging copy.
    treg = time.perf_counter()
    cio.host_register(host)
    reg_ms = (time.perf_counter() - treg) * 1e3
    try:
        for _ in range(max(1, args.warmup)):
            out_reg = cio.crc32_batch_host_packed(host, offs, lens)
        barrier(dist)
        t0 = time.perf_counter()
        for _ in range(steps):
            out_reg = cio.crc32_batch_host_packed(host, offs, lens)
        barrier(dist)
        elapsed_reg = max_over_ranks(time.perf_counter() - t0, dist, device)
        legs_reg = cio.pipe_last_timing()
        # the DMA engine's rate from the registered pages themselves (the
        # registered path's ceiling), beside pinned_h2d_GBps in `breakdown`
        import ctypes
        f_h2d = cio.lib().cioa_debug_h2d_gbps
        f_h2d.restype = ctypes.c_double
        f_h2d.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        reg_h2d = round(f_h2d(host.ctypes.data, host.size, 5), 2)
    finally:
        cio.host_unregister(host)
    value_reg = int(lens.sum()) * world * steps / elapsed_reg / 1e9
    check = {"registered_equals_staged": bool(np.array_equal(out, out_reg))}
    host_cpu = host_cpu_batch(host, offs, lens, out)
    if world == 1:
        import hashlib
        with open(os.path.join(ROOT, "tests", "golden", "crc32_vectors.json")) as f:
            g = json.load(f)["cfg2"]
        check["golden_sha256_match"] = hashlib.sha256(
            np.asarray(out, dtype="<u4").tobytes()).hexdigest() == g["sha256_of_raw_le"]
    return {"metric": "end-to-end CRC32 GB/s from host memory (pinned staging + H2D + kernel + D2H)",
            "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / steps * 1e3, 4),
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "u8",
            "data": "synthetic, pageable host memory", "config": desc,
            "staged_call_ms": {"min": round(min(call_s) * 1e3, 3), "median": round(float(np.median(call_s)) * 1e3, 3),
                               "max": round(max(call_s) * 1e3, 3)},
            "registered_in_place": {"value": round(value_reg, 3), "unit": "GB/s",
                                    "ms_per_step": round(elapsed_reg / steps * 1e3, 4),
                                    "register_ms_once": round(reg_ms, 2),
                                    "h2d_from_registered_pages_GBps": reg_h2d,
                                    "note": "host batch pinned once with cio_crc32_host_register "
                                            "(outside the timed loop); chunks DMA'd directly"},
            "host_cpu_batch": host_cpu,
            "numa": {**numa_info(device.index or 0, host), "bound_cpus": bound},
            "breakdown": e2e_breakdown(host, device),
            "pipe_legs_last_call": {"staged": legs_staged, "registered": legs_reg,
                                    "note": "cio_gpu_pipe_last_timing() after the last timed call: total = the "
                                            "library's wall time for the batch; copy = host copy into pinned "
                                            "staging (caller's view, overlapped with the DMA of earlier "
                                            "groups); slot_wait = waiting for a staging slot to drain; "
                                            "total minus the DMA bound (bytes / pinned_h2d_GBps) is "
                                            "pipeline fill/drain and host overhead"},
            "check": check}


def page_node(addr):
    """NUMA node of the page at addr (get_mempolicy MPOL_F_NODE|MPOL_F_ADDR), or -1."""
    import ctypes
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        node = ctypes.c_int(-1)
        rc = libc.syscall(239, ctypes.byref(node), None, ctypes.c_ulong(0), ctypes.c_void_p(addr),
                          ctypes.c_ulong(3))
        return node.value if rc == 0 else -1
    except (OSError, AttributeError):
        return -1


def numa_info(dev_index, host=None):
    """Where the host legs run: the GPU's NUMA node, the nodes of the host
    batch's first and middle pages, and the CPUs this process may use."""
    import chunkio_amd as cio
    info = {"gpu_node": int(cio.lib().cio_gpu_numa_node(dev_index))}
    try:
        with open("/sys/devices/system/node/online") as f:
            info["nodes_online"] = f.read().strip()
    except OSError:
        pass
    if host is not None:
        info["host_batch_nodes"] = [page_node(host.ctypes.data), page_node(host.ctypes.data + host.size // 2)]
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    return info


def bind_to_gpu_node(dev_index):
    """Restrict this process to the GPU's NUMA node before the host batch is
    allocated, as a deployment binds each rank to its GPU's socket (the host
    legs' pages and threads then sit next to the PCIe link they feed).
    CIO_BENCH_NUMA_BIND=0 leaves the affinity alone.  Returns the number of
    CPUs bound to, or None."""
    if os.environ.get("CIO_BENCH_NUMA_BIND") == "0":
        return None
    import chunkio_amd as cio
    node = int(cio.lib().cio_gpu_numa_node(dev_index))
    if node < 0:
        return None
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            cpus = set()
            for part in f.read().strip().split(","):
                a, _, b = part.partition("-")
                cpus.update(range(int(a), int(b or a) + 1))
        cpus &= os.sched_getaffinity(0)
        if cpus:
            os.sched_setaffinity(0, cpus)
            return len(cpus)
    except (OSError, ValueError):
        pass
    return None


def host_cpu_threads():
    """Host threads for the library's host CRC legs: the box's CPU share per
    GPU (16 on the MI355X box), at most this process's affinity."""
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    return max(1, min(16, share))


def host_cpu_batch(host, offs, lens, gpu_out):
    """The library's own host path over the same host batch (cio_crc32_batch_cpu:
    crc_update with VPCLMULQDQ folding, 1 thread and the box's per-GPU CPU
    share), next to the GPU host paths: which engine wins for host-resident
    chunks (crc_route.c routes the chunk layer by this)."""
    import chunkio_amd as cio
    res = {}
    for t in sorted({1, host_cpu_threads()}):
        cio.crc32_batch_cpu_packed(host, offs, lens, threads=t)          # warm (pool, pages)
        reps = 3 if t == 1 else 10
        t0 = time.perf_counter()
        for _ in range(reps):
            got = cio.crc32_batch_cpu_packed(host, offs, lens, threads=t)
        dt = (time.perf_counter() - t0) / reps
        res[f"threads_{t}"] = {"GBps": round(int(lens.sum()) / dt / 1e9, 2), "ms": round(dt * 1e3, 3),
                               "equals_gpu": bool(np.array_equal(got, gpu_out))}
    res["note"] = ("cio_crc32_batch_cpu over the same pageable host batch (DRAM-resident), min of "
                   "back-to-back calls' mean; no PCIe")
    return res


def e2e_breakdown(host, device):
    """Ceilings of the two host-side legs on this box: pinned H2D DMA and host memcpy."""
    import torch
    n = host.size
    src = torch.from_numpy(host)
    pinned = torch.empty(n, dtype=torch.uint8).pin_memory()
    dev = torch.empty(n, dtype=torch.uint8, device=device)
    dev.copy_(pinned, non_blocking=True)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(5):
        dev.copy_(pinned, non_blocking=True)
    torch.cuda.synchronize(device)
    h2d = 5 * n / (time.perf_counter() - t0) / 1e9
    pinned.copy_(src)
    t0 = time.perf_counter()
    for _ in range(3):
        pinned.copy_(src)
    cp = 3 * n / (time.perf_counter() - t0) / 1e9
    return {"pinned_h2d_GBps": round(h2d, 2), "host_to_pinned_copy_GBps_torch": round(cp, 2),
            "torch_threads": torch.get_num_threads()}


def run_perf(args, rank, world, device, dist, compact=False):
    """BASELINE config 1's loop (`tools/cio -k -p 400kb.txt`: 1000 files x 5 x
    409600 B with CRC32) through the C chunk layer (cioa_bench_perf_write,
    include/chunkio_amd/cioa_chunk.h): appends only copy (CIOA_DEFERRED_CRC)
    and the chunks are synced 100 at a time through ONE GPU pass each
    (cioa_chunk_sync_batch).  Host memory end to end, files on the box's /tmp.
    Beside it: the same C layer in the reference's order (crc_update per write
    on the CPU, `c_layer_immediate`), and the reference loop itself
    (oracle/_ref: the reference's own crc_update under the restated loop),
    with and without the CRC."""
    import ctypes
    import shutil
    from chunkio_amd import chunkfile as cf
    d400 = np.fromfile(os.path.join(ROOT, "tests", "golden", "400kb.txt"), dtype=np.uint8).tobytes()
    files, writes, batch = 1000, 5, 100
    reps = max(1, min(args.steps, 3))
    if compact:
        # the default line's leg: the deferred C layer only, one warm pass +
        # `reps` timed; the reference loop is cpu_baseline.cio_perf_k_p there
        reps = max(1, min(args.steps, 2))

    def timed(flags, tag):
        times = []
        hdr_ok = True
        root = tempfile.mkdtemp(prefix=f"cioa-perf-{tag}-")
        try:
            for r in range(reps + 1):                  # first pass warms the GPU pipeline / page cache
                path = os.path.join(root, f"run{r}")
                secs, nb = cf.perf_write(path, d400, files, writes, batch, flags)
                if r:
                    times.append(secs)
                with open(os.path.join(path, "test-perf", "perf-test-0999.txt"), "rb") as f:
                    hdr_ok &= f.read(10).hex() == "c100088740e700000000"
                shutil.rmtree(path)
        finally:
            shutil.rmtree(root, ignore_errors=True)
        return min(times), nb, hdr_ok

    t_def, nbytes, ok_def = timed(cf.CIO_CHECKSUM | cf.CIOA_DEFERRED_CRC, "deferred")
    # the same with each batch's CRC pass on its own thread while the next
    # batch is written (cioa_chunk_sync_batch_begin / _end)
    t_pipe, _, ok_pipe = timed(cf.CIO_CHECKSUM | cf.CIOA_DEFERRED_CRC | cf.CIOA_BENCH_PIPELINED_SYNC, "pipelined")
    pipelined = {"GBps": round(nbytes / t_pipe / 1e9, 3), "ms": round(t_pipe * 1e3, 2),
                 "note": "deferred CRC, each 100-chunk sync batch's pass (default route) overlapping the next "
                         "batch's writes: cioa_chunk_sync_batch_begin / _end"}
    # The same C layer in the reference's order (crc_update per write on the
    # calling thread: VPCLMULQDQ folding over the cached 400 KB buffer), and
    # deferred with the sync batches on the host (host threads granted, so the
    # route puts them on the CPU pool): the library's own host paths beside
    # the GPU sync, same run.
    import chunkio_amd as cio
    t_imm, _, ok_imm = timed(cf.CIO_CHECKSUM, "immediate")
    nt = host_cpu_threads()
    try:
        cio.route(reset=True, threads=nt)
        t_dh, _, ok_dh = timed(cf.CIO_CHECKSUM | cf.CIOA_DEFERRED_CRC, "deferred-host")
    finally:
        cio.route(reset=True)
    host_paths = {"c_layer_immediate": {"GBps": round(nbytes / t_imm / 1e9, 3), "ms": round(t_imm * 1e3, 2),
                                        "threads": 1,
                                        "note": "crc_update per write on the calling thread (reference order), "
                                                "finalize per sync"},
                  f"c_layer_deferred_host_{nt}t": {"GBps": round(nbytes / t_dh / 1e9, 3), "ms": round(t_dh * 1e3, 2),
                                                    "threads": nt,
                                                    "note": "appends only copy; each 100-chunk sync batch CRC'd by "
                                                            "cio_crc32_batch_cpu on the host pool"}}
    if compact:
        return {"metric": "cio -k -p loop (1000 files x 5 x 400 KB, CRC32) GB/s with deferred CRC + batched "
                          "GPU sync", "value": round(nbytes / t_def / 1e9, 3), "unit": "GB/s", "steps": reps,
                "warmup": 1, "ms_per_step": round(t_def * 1e3, 2), "scaling": "weak",
                "vs_baseline": round(nbytes / t_def / 545_507_660, 2),
                "vs_baseline_note": "BASELINE.md's published `cio -k -p` rate, 545,507,660 B/s (README.md:120-129, "
                                    "hardware unstated)",
                "config": {"workload": "config 1 loop through the C chunk layer (cioa_bench_perf_write): open, "
                                       "5 x write 409600 B, sync (batches of 100 chunks per GPU pass), close",
                           "files": files, "writes": writes, "sync_batch": batch},
                "pipelined_sync": pipelined, "host_paths": host_paths,
                "check": {"last_file_header_c100088740e7": bool(ok_def and ok_imm and ok_dh and ok_pipe)},
                "cpu_baseline_ref": "cpu_baseline.cio_perf_k_p of this line: the reference loop with the "
                                    "reference's own crc_update, same box, same run"}
    from oracle import pyoracle as po
    lib = po.ref()
    kind, prefix = "reference", "ref_"
    if lib is None:
        lib, kind, prefix = po.oracle(), "port", "oracle_"
    buf = np.frombuffer(d400, np.uint8)
    ref = {}
    for ck in (1, 0):
        with tempfile.TemporaryDirectory(prefix="cioa-perf-") as tmp:
            nb = ctypes.c_uint64(0)
            secs = getattr(lib, prefix + "cio_perf_write")(tmp.encode(), buf.ctypes.data, buf.size,
                                                           files, writes, ck, ctypes.byref(nb))
            ref["crc_on" if ck else "crc_off"] = {"seconds": round(secs, 4),
                                                   "GBps": round(nb.value / secs / 1e9, 3)}
    return {"metric": "cio -k -p loop (1000 files x 5 x 400 KB, CRC32) GB/s with deferred CRC + batched GPU sync",
            "value": round(nbytes / t_def / 1e9, 3), "unit": "GB/s", "n_gpus": 1, "steps": reps, "warmup": 1,
            "ms_per_step": round(t_def * 1e3, 2), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(nbytes / t_def / 545_507_660, 2), "dtype": "u8",
            "data": "tests/golden/400kb.txt (the reference's perf input)",
            "config": {"workload": "config 1 loop through the C chunk layer (cioa_bench_perf_write): open, "
                                   "5 x write 409600 B, sync (batches of 100 chunks per GPU pass), close",
                       "files": files, "writes": writes, "sync_batch": batch},
            "pipelined_sync": pipelined, "host_paths": host_paths,
            "check": {"last_file_header_c100088740e7": bool(ok_def and ok_imm and ok_dh and ok_pipe)},
            "vs_baseline_note": "BASELINE.md's published `cio -k -p` rate, 545,507,660 B/s (README.md:120-129, "
                                "hardware unstated)",
            "cpu_baseline": {"value": ref["crc_on"]["GBps"], "unit": "GB/s", "cores": 1, "kind": kind,
                             "sample": "the same loop in C with crc_update per write (1 thread)",
                             "crc_off_GBps": ref["crc_off"]["GBps"], **cpu_info()}}


def make_perf_files(root, files=1000, bad=500):
    """The 1000 chunk files `tools/cio -k -p` leaves (2,068,480 B each: header,
    5 x 400kb.txt, CRC 0x088740E7), written once through the chunk layer and
    copied, with a flipped content byte in file `bad`."""
    import shutil
    from chunkio_amd import chunkfile as cf
    d400 = np.fromfile(os.path.join(ROOT, "tests", "golden", "400kb.txt"), dtype=np.uint8).tobytes()
    paths = [os.path.join(root, f"perf-test-{i:04d}.txt") for i in range(files)]
    c, _ = cf.ChunkFile.open(paths[0], deferred_crc=True)
    for _ in range(5):
        c.write(d400)
    cf.sync_batch([c])
    c.close()
    for p in paths[1:]:
        shutil.copyfile(paths[0], p)
    with open(paths[bad], "r+b") as f:
        f.seek(24 + 123456)
        b = f.read(1)
        f.seek(24 + 123456)
        f.write(bytes([b[0] ^ 0x20]))
    return paths


def run_verify(args, rank, world, device, dist, compact=False):
    """batched verify-on-load of a stream directory.  1000
    chunk files as `tools/cio -k -p` leaves them (2,068,480 B each: header,
    5 x 400kb.txt, CRC 0x088740E7; one of them with a flipped content byte)
    on the box's /tmp (page cache), verified by ONE cio_verify_paths call
    (open + header/length checks + pread of the CRC regions into the GPU
    pipeline + one batched GPU CRC pass + 8-byte compare + close).  Beside it, the reference's per-file verify
    (cio_file_format_check, src/cio_file.c:266-290: crc_update over
    [22, 24 + meta + content) then compare) with the reference's own
    crc_update (oracle/_ref), single thread, over the same mapped files."""
    import shutil
    from chunkio_amd import chunkfile as cf
    d400 = np.fromfile(os.path.join(ROOT, "tests", "golden", "400kb.txt"), dtype=np.uint8).tobytes()
    files, bad = 1000, 500
    reps = max(1, min(args.steps, 10))
    ncpu = 100 if compact else 200
    root = tempfile.mkdtemp(prefix="cioa-verify-")
    try:
        paths = make_perf_files(root, files, bad)
        fsize = os.path.getsize(paths[0])
        region = 2 + 5 * len(d400)              # [22, 24 + meta_len + content_len)
        for _ in range(max(1, args.warmup)):
            st, er, cr = cf.verify_paths(paths)
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            st, er, cr = cf.verify_paths(paths)
            times.append(time.perf_counter() - t0)
        t = min(times)
        ok_idx = [i for i in range(files) if i != bad]
        check = {"good_files_ok": bool(np.all(st[ok_idx] == 0)),
                 "good_crc_088740e7": bool(np.all((cr[ok_idx] ^ 0xFFFFFFFF) == 0x088740E7)),
                 "flipped_file_bad_checksum": bool(st[bad] == -3 and er[bad] == -10)}
        # The same call with the CRC pass on the host (crc_route.c): one
        # thread (every batch forced to the host) and the box's per-GPU CPU
        # share (host threads granted: the route's model puts every
        # host-memory batch on the CPU).
        import chunkio_amd as cio
        host_route = {}
        try:
            # `value` is the default route: GPU-bound batches split with the
            # calling thread (crc_route.c); gpu_alone is the same call with
            # the split route off (every CRC byte on the GPU).
            nt = host_cpu_threads()
            for tag, kw in (("gpu_alone", {"split": False}), ("threads_1", {"cpu_max": -1, "threads": 1}),
                            (f"threads_{nt}", {"cpu_max": -1, "threads": nt}),
                            (f"default_route_threads_{nt}", {"threads": nt})):
                cio.route(reset=True, **kw)
                cf.verify_paths(paths)
                ht = []
                for _ in range(reps):
                    t0 = time.perf_counter()
                    st2, er2, cr2 = cf.verify_paths(paths)
                    ht.append(time.perf_counter() - t0)
                host_route[tag] = {"GBps": round(files * region / min(ht) / 1e9, 3),
                                   "ms": round(min(ht) * 1e3, 3),
                                   "same_results_as_gpu": bool(np.array_equal(st2, st) and np.array_equal(er2, er)
                                                               and np.array_equal(cr2, cr))}
        finally:
            cio.route(reset=True)
        host_route["note"] = ("cio_verify_paths with the CRC batch routed to the library's host crc_update "
                              "(cio_crc32_batch_fd_cpu: pread + VPCLMULQDQ folding) instead of the GPU; "
                              "gpu_alone: the GPU without the split route's host share; default_route_threads_N: "
                              "the default route with N host threads (the split route shares the batch with "
                              "the GPU while the host is < 3x faster than it)")
        cpu = None
        if rank == 0 and not args.no_cpu:
            import mmap
            from oracle import pyoracle as po
            lib, kind = po.ref(), "reference"
            fn = "crc_update"
            if lib is None:
                lib, kind, fn = po.oracle(), "port", "oracle_crc_update"
            f_upd = getattr(lib, fn)
            t0 = time.perf_counter()
            nbad = 0
            for p in paths[:ncpu]:
                with open(p, "rb") as f:
                    m = mmap.mmap(f.fileno(), 0, prot=mmap.PROT_READ)
                    a = np.frombuffer(m, dtype=np.uint8)
                    crc = int(f_upd(0xFFFFFFFF, a.ctypes.data + 22, region)) ^ 0xFFFFFFFF
                    nbad += int(a[2:6].tobytes() != crc.to_bytes(4, "big"))
                    del a
                    m.close()
            tc = time.perf_counter() - t0
            cpu = {"value": round(ncpu * region / tc / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": kind,
                   "sample": f"first {ncpu} of the same files: open + mmap + crc_update over the region + "
                             "4-byte compare, one thread", "bad_found_in_sample": nbad}
    finally:
        shutil.rmtree(root, ignore_errors=True)
    res = {"metric": "batched verify-on-load GB/s (1000 chunk files from page cache, one cio_verify_paths call)",
           "value": round(files * region / t / 1e9, 3), "unit": "GB/s", "n_gpus": 1, "steps": reps,
           "warmup": args.warmup, "ms_per_step": round(t * 1e3, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8",
           "data": "tests/golden/400kb.txt x 5 per file (the reference's perf-test files)",
           "config": {"workload": "verify-on-load of 1000 x 2,068,480-B chunk files (CRC region "
                                  f"{region} B each), open/pread/close included", "files": files,
                      "file_bytes": fsize},
           "host_route": host_route,
           "check": check}
    if cpu is not None:
        res["cpu_baseline"] = cpu
    return res


def multi_device_list(world, visible, rehearse):
    """Device entries for the all-devices leg: 0..N-1, or -- rehearsing N
    ranks on fewer GPUs -- the visible ones round-robin (shared: True).
    None when the GPUs are too few and this is not a rehearsal."""
    if visible >= world:
        return list(range(world)), False
    if not rehearse or visible < 1:
        return None, True
    return [i % visible for i in range(world)], True


def node_cpus(node):
    """CPUs of a NUMA node (sysfs cpulist), empty when unknown."""
    cpus = set()
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            for part in f.read().strip().split(","):
                a, _, b = part.partition("-")
                cpus.update(range(int(a), int(b or a) + 1))
    except (OSError, ValueError):
        pass
    return cpus


def _multi_device_host(args, world, device):
    """Rank 0's half of multi_device_host_leg (see there)."""
    import hashlib
    import shutil
    import torch
    import chunkio_amd as cio
    from chunkio_amd import chunkfile as cf
    from chunkio_amd import workloads as wl
    rehearse = os.environ.get("CIO_BENCH_REHEARSE") == "1"
    devices, shared = multi_device_list(world, torch.cuda.device_count(), rehearse)
    if devices is None:
        return {"error": f"{world} devices wanted, {torch.cuda.device_count()} visible"}
    if ORIG_AFFINITY:
        os.sched_setaffinity(0, ORIG_AFFINITY)       # undo the per-GPU NUMA binding of the e2e leg
    res = {"devices": devices, "shared_devices_rehearsal": shared}
    # -- (1) the weak cfg2 job of N GPUs (N x 1024 x 409,600 B) in pageable host
    #    memory, one cio_crc32_batch_host_multi call: chunk k -> devices[k % N]
    n = wl.CFG2_N * world
    lens = np.full(n, wl.CFG2_LEN, dtype=np.uint64)
    offs = wl.packed_offsets(lens, align=16)
    total = int(lens.sum())
    gen = torch.empty(wl.batch_bytes(offs, lens) + 16, dtype=torch.uint8, device=device)
    cio.fill_synthetic(gen, offs, lens, wl.CFG2_SEED, ids=np.arange(n, dtype=np.uint64))
    host = gen.cpu().numpy()
    del gen
    torch.cuda.empty_cache()
    out = cio.crc32_batch_host_packed(host, offs, lens, devices=devices)        # warm: pipelines, pools
    reps = max(1, min(args.steps, 5))
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = cio.crc32_batch_host_packed(host, offs, lens, devices=devices)
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    # the same batch pinned in place once (long-lived chunk mappings): every
    # device's DMA engine reads the caller's pages, no staging copy
    t0 = time.perf_counter()
    cio.host_register(host)
    reg_ms = (time.perf_counter() - t0) * 1e3
    try:
        out_reg = cio.crc32_batch_host_packed(host, offs, lens, devices=devices)
        tr = []
        for _ in range(reps):
            t0 = time.perf_counter()
            out_reg = cio.crc32_batch_host_packed(host, offs, lens, devices=devices)
            tr.append(time.perf_counter() - t0)
    finally:
        cio.host_unregister(host)
    want = weak_job_golden("cfg2", world)
    per_dev = {}
    for k, d in enumerate(devices):
        per_dev.setdefault(str(d), 0)
        per_dev[str(d)] += int(lens[k::len(devices)].sum())
    numa = {}
    for d in sorted(set(devices)):
        node = int(cio.lib().cio_gpu_numa_node(d))
        local = node_cpus(node) & (ORIG_AFFINITY or set()) if node >= 0 else set()
        numa[str(d)] = {"numa_node": node, "node_cpus_in_affinity": len(local),
                        "copy_threads": min(15, max(0, (os.cpu_count() or 1) - 1)) + 1,   # CopyPool + caller
                        "copy_threads_pinned_to_node": bool(local)}
    host_cpu = {}
    try:
        nproc = len(os.sched_getaffinity(0))
    except AttributeError:
        nproc = os.cpu_count() or 1
    for tn in sorted({16, min(64, nproc)}):
        cio.crc32_batch_cpu_packed(host, offs, lens, threads=tn)
        tt = []
        for _ in range(3):
            t0 = time.perf_counter()
            got = cio.crc32_batch_cpu_packed(host, offs, lens, threads=tn)
            tt.append(time.perf_counter() - t0)
        host_cpu[f"threads_{tn}"] = {"GBps": round(total / min(tt) / 1e9, 2), "ms": round(min(tt) * 1e3, 3),
                                     "equals_gpu": bool(np.array_equal(got, out))}
    host_cpu["note"] = (f"cio_crc32_batch_cpu over the same host batch (16 threads, and this process's CPUs "
                        f"up to the pool's 64: {nproc} in affinity)")
    res["host_batch_multi"] = {
        "call": "cio_crc32_batch_host_multi (staged: copy pools -> pinned staging -> H2D -> kernel, "
                "every device's pipeline concurrently)",
        "GBps": round(total / t / 1e9, 3), "ms": round(t * 1e3, 3), "bytes": total, "chunks": n,
        "per_device_GBps": round(total / t / 1e9 / len(set(devices)), 3),
        "registered_in_place": {"GBps": round(total / min(tr) / 1e9, 3), "ms": round(min(tr) * 1e3, 3),
                                "register_ms_once": round(reg_ms, 2),
                                "equals_staged": bool(np.array_equal(out_reg, out))},
        "bytes_per_device": per_dev, "numa_per_device": numa, "reps": reps,
        "host_batch_page_nodes": [page_node(host.ctypes.data + host.size * q // 4) for q in range(4)],
        "check": {"golden_sha256_match_full_job": (hashlib.sha256(np.asarray(out, dtype="<u4").tobytes())
                                                   .hexdigest() == want) if want else None},
        "host_cpu_batch": host_cpu}
    del host
    # -- (2) verify-on-load of the 1000 perf files with devices[] (file ranges
    #    pread by each device's copy pool; cio_verify_paths_multi)
    root = tempfile.mkdtemp(prefix="cioa-multi-")
    try:
        files, bad = 1000, 500
        paths = make_perf_files(root, files, bad)
        region = 2 + 5 * 409600
        ok_idx = [i for i in range(files) if i != bad]
        legs = {}
        nt = host_cpu_threads()
        try:
            for tag, kw in (("gpus_alone", {"cpu_max": 0}), ("default_route", {}),
                            (f"host_threads_{nt}", {"cpu_max": -1, "threads": nt})):
                cio.route(reset=True, **kw)
                cf.verify_paths(paths, devices=devices)
                vt = []
                for _ in range(3):
                    t0 = time.perf_counter()
                    st, er, cr = cf.verify_paths(paths, devices=devices)
                    vt.append(time.perf_counter() - t0)
                legs[tag] = {"GBps": round(files * region / min(vt) / 1e9, 3), "ms": round(min(vt) * 1e3, 3),
                             "check": bool(np.all(st[ok_idx] == 0)
                                           and np.all((cr[ok_idx] ^ 0xFFFFFFFF) == 0x088740E7)
                                           and st[bad] == -3 and er[bad] == -10)}
        finally:
            cio.route(reset=True)
        legs["note"] = ("one cio_verify_paths_multi call over 1000 x 2,068,480-B files in the page cache; "
                        "gpus_alone: every CRC byte on the devices (threshold 0); default_route: the "
                        "route as shipped (one host CRC thread, split route on); host_threads_N: every "
                        "batch on N host threads, no GPU")
        res["verify_paths_multi"] = legs
    finally:
        shutil.rmtree(root, ignore_errors=True)
    return res


def multi_device_host_leg(args, rank, world, device, dist, runner=None):
    """How ONE chunkio process would use every GPU of the node for chunks in
    host memory (Fluent Bit is one process: src/cio_scan.c:39-125 loads every
    stream in it): after the per-rank legs, rank 0 alone -- the other ranks
    wait at a barrier -- calls the library's single-process multi-device API
    with devices = 0..N-1: cio_crc32_batch_host_multi over the whole weak cfg2
    job of N GPUs (N x 1024 x 409,600 B, checked against its reference digest)
    and cio_verify_paths_multi over the 1000 perf files; beside them the host's
    own CRC over the same batch on 16 threads and on the process's CPUs.  At
    N = 1 it is the e2e and verify legs again on device 0.  Returns rank 0's
    result (None on the other ranks)."""
    barrier(dist)
    res = None
    if rank == 0:
        t0 = time.perf_counter()
        res = (runner or _multi_device_host)(args, world, device)
        res["wall_s"] = round(time.perf_counter() - t0, 2)
    barrier(dist)
    return res


def diagnostic_batches(device):
    """SURVEY §8(d)'s two extra cfg2-shaped batches, single buffer, 50
    back-to-back launches under one event pair: 400kb.txt tiled 1024 times
    (every CRC must finalize to 0x777A8F30) and an all-zero batch (the LDS
    tables' best case; checked against zlib)."""
    import zlib
    import torch
    import chunkio_amd as cio
    from chunkio_amd import workloads as wl
    d400 = np.fromfile(os.path.join(ROOT, "tests", "golden", "400kb.txt"), dtype=np.uint8)
    n, ln = wl.CFG2_N, wl.CFG2_LEN
    offs = np.arange(n, dtype=np.uint64) * np.uint64(ln)
    lens = np.full(n, ln, dtype=np.uint64)
    plan = cio.Crc32Plan(offs, lens)
    lib = cio.lib()
    stream = torch.cuda.current_stream(device)
    sptr = int(stream.cuda_stream)
    out = torch.empty(n, dtype=torch.int32, device=device)
    res = {}
    for name, buf, want in (
            ("tiled_400kb", torch.from_numpy(np.tile(d400, n)).to(device), 0x777A8F30),
            ("all_zero", torch.zeros(n * ln, dtype=torch.uint8, device=device),
             zlib.crc32(bytes(ln)))):
        t0 = time.perf_counter()                 # device ramp, as in run_crc
        while time.perf_counter() - t0 < 0.15:
            for _ in range(16):
                plan.exec(buf, out, stream=stream)
            torch.cuda.synchronize(device)
        e0, e1 = lib.cio_gpu_event_create(), lib.cio_gpu_event_create()
        lib.cio_gpu_event_record(e0, sptr)
        for _ in range(50):
            plan.exec(buf, out, stream=stream)
        lib.cio_gpu_event_record(e1, sptr)
        torch.cuda.synchronize(device)
        ms = lib.cio_gpu_event_elapsed_ms(e0, e1) / 50
        lib.cio_gpu_event_destroy(e0)
        lib.cio_gpu_event_destroy(e1)
        got = out.cpu().numpy().view(np.uint32) ^ np.uint32(0xFFFFFFFF)
        res[name] = {"GBps": round(n * ln / (ms * 1e-3) / 1e9, 1), "kernel_ms_mean": round(ms, 5),
                     "all_crc_match": bool(np.all(got == np.uint32(want))), "want": f"0x{want:08x}",
                     "note": "one buffer (no rotation); diagnostic, not the headline"}
        del buf
    plan.close()
    torch.cuda.empty_cache()
    return res


def other_chunk_sizes(args, rank, world, device, dist):
    """The north star's 4 KiB and 4 MiB chunk batches measured in the same run
    (same process layout, same N), so every scaling run reports all three
    chunk sizes: cfg4k (102 400 x 4 KiB per GPU, weak) and cfg4 (8192 x 4 MiB
    per job, strong).  Same timing method as the headline line."""
    import copy
    import torch
    out = {}
    sizes = (("cfg4k", 200, 50), ("cfg4", 20, 5))
    if os.environ.get("CIO_BENCH_SIZES") is not None:
        # diagnostic: a subset of the sizes (e.g. "" for none, "cfg4k")
        sizes = tuple(x for x in sizes if x[0] in os.environ["CIO_BENCH_SIZES"].split(","))
    for cfg, steps, warm in sizes:
        torch.cuda.empty_cache()
        a = copy.copy(args)
        a.config, a.steps, a.warmup, a.no_cpu = cfg, steps, warm, True
        a.no_cpu_sample = args.no_cpu
        r = run_crc(a, rank, world, device, dist)
        out[cfg] = {"value": r["value"], "unit": r["unit"], "scaling": r["scaling"], "steps": steps,
                    "warmup": warm, "ms_per_step": r["ms_per_step"], "workload": r["config"]["workload"],
                    "roofline": {k: r["roofline"][k] for k in ("achieved", "peak", "frac", "kernel",
                                                                "kernel_ms_mean", "traffic", "workgroups",
                                                                "frac_of_read_stream")},
                    "check": r.get("check", {})}
        if "cpu_baseline" in r:
            out[cfg]["cpu_baseline"] = r["cpu_baseline"]
        if "per_gpu" in r:
            out[cfg]["per_gpu"] = r["per_gpu"]
    torch.cuda.empty_cache()
    return out


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def visible_gpus():
    """GPUs this process could use, counted WITHOUT touching the GPU: the KFD
    topology in sysfs (nodes with SIMDs) whose DRM render node this process
    may open (a container can list every GPU of the host in sysfs but hold
    only some render nodes), narrowed by the *_VISIBLE_DEVICES lists the
    runtime honours.  Returns (count, how)."""
    import glob
    n = 0
    for prop in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(prop) as f:
                kv = dict(line.split(None, 1) for line in f if line.strip())
        except (OSError, ValueError):
            continue
        if int(kv.get("simd_count", "0")) <= 0:
            continue
        minor = kv.get("drm_render_minor", "").strip()
        if minor and not os.access(f"/dev/dri/renderD{minor}", os.R_OK | os.W_OK):
            continue
        n += 1
    how = "kfd-sysfs+render-node-access"
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
            how += f"+{var}"
    return n, how


def runtime_gpu_count():
    """torch.cuda.device_count() in a child process (0 if that fails)."""
    import subprocess
    try:
        r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                           capture_output=True, text=True, timeout=600)
        return int(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else 0
    except (OSError, ValueError, IndexError, subprocess.TimeoutExpired):
        return 0


def spawn_ranks(args):
    """`python bench.py --gpus N` with no launcher environment: start N rank
    processes of this script (one per GPU, the layout torch.distributed.run
    gives) and exit with the worst child status.  Nothing here touches the GPU
    (the devices are counted from sysfs, torch is not imported), so the
    children start from a clean process."""
    import subprocess
    visible, _ = visible_gpus()
    rehearse = os.environ.get("CIO_BENCH_REHEARSE") == "1" or os.environ.get("CIO_BENCH_SHARE_DEVICES") == "1"
    if visible < args.gpus and not rehearse:
        # A sysfs layout this count does not know could under-count: ask the
        # runtime in a child process (this one stays clean for the ranks).
        visible = max(visible, runtime_gpu_count())
    if visible < args.gpus and not rehearse:
        print(f"bench.py: --gpus {args.gpus} but only {visible} GPU(s) visible", file=sys.stderr)
        return 2
    import signal
    env = dict(os.environ, WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    procs = []

    def stop_all(grace_s=10.0):
        """SIGTERM every live rank, then SIGKILL what is left after grace_s."""
        live = [p for p in procs if p.poll() is None]
        for p in live:
            p.terminate()
        deadline = time.monotonic() + grace_s
        for p in live:
            try:
                p.wait(timeout=max(0.1, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    def on_signal(signum, _frame):
        stop_all()
        sys.exit(128 + signum)

    old_handlers = {sig: signal.signal(sig, on_signal) for sig in (signal.SIGTERM, signal.SIGINT)}
    try:
        for r in range(args.gpus):
            e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=e))
            print(f"bench.py: rank {r} pid {procs[-1].pid}", file=sys.stderr, flush=True)
        # Poll every rank (not in order): the first non-zero exit ends the job,
        # so a rank that dies at init or mid-run cannot leave its siblings
        # blocked in a barrier until the gloo timeout.
        while True:
            rcs = [p.poll() for p in procs]
            bad = [(r, rc) for r, rc in enumerate(rcs) if rc is not None and rc != 0]
            if bad:
                r, rc = bad[0]
                print(f"bench.py: rank {r} exited with status {rc}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                stop_all()
                return rc if rc > 0 else 128 - rc
            if all(rc == 0 for rc in rcs):
                return 0
            time.sleep(0.1)
    finally:
        stop_all()
        for sig, h in old_handlers.items():
            signal.signal(sig, h)


def other_configs(args, rank, world, device, dist, only=None):
    """The north star's other single-GPU workloads, short runs in the same
    process so the default line carries every config: cfg3 (65,536 mixed
    4 KB-4 MB chunks, ~39.7 GB, persistent load-balanced kernel), cfg5 (SHA-1
    over the cfg2 batch) and the end-to-end host path (staged and registered
    in place).  Each entry is the full line of that --config, trimmed."""
    import copy
    import torch
    out = {}
    t0 = time.perf_counter()
    legs = [("cfg3", 5, 2), ("sha1", 10, 2), ("e2e", 30, 10)]
    if world == 1:
        # SURVEY §8(f) rows 1 and 3 (host-side, one process): batched
        # verify-on-load of 1000 chunk files, and the config-1 loop through
        # the C chunk layer with deferred CRC + batched GPU sync.
        legs += [("verify", 3, 1), ("perf", 2, 1)]
    if only is not None:
        legs = [leg for leg in legs if leg[0] in only]
    if os.environ.get("CIO_BENCH_LEGS"):
        # diagnostic: a subset / order of the legs (e.g. "e2e,cfg3")
        by = {cfg: (cfg, s, w) for cfg, s, w in legs}
        legs = [by[c] for c in os.environ["CIO_BENCH_LEGS"].split(",") if c in by]
    for cfg, steps, warm in legs:
        torch.cuda.empty_cache()
        a = copy.copy(args)
        a.config, a.steps, a.warmup = cfg, steps, warm
        a.no_cpu = cfg not in ("verify", "sha1") or args.no_cpu
        a.no_cpu_sample = args.no_cpu
        t1 = time.perf_counter()
        if cfg == "sha1":
            r = run_sha1(a, rank, world, device, dist)
        elif cfg == "e2e":
            r = run_e2e(a, rank, world, device, dist)
        elif cfg == "verify":
            r = run_verify(a, rank, world, device, dist, compact=True)
        elif cfg == "perf":
            r = run_perf(a, rank, world, device, dist, compact=True)
        else:
            r = run_crc(a, rank, world, device, dist)
        keep = {k: r[k] for k in ("metric", "value", "unit", "scaling", "steps", "warmup", "ms_per_step")}
        keep["workload"] = r["config"].get("workload")
        for k in ("roofline", "check", "per_gpu", "registered_in_place", "breakdown", "pipe_legs_last_call",
                  "host_cpu_batch", "host_route", "host_paths", "pipelined_sync", "numa", "staged_call_ms",
                  "cpu_baseline", "cpu_baseline_ref", "vs_baseline", "vs_baseline_note"):
            if k in r:
                keep[k] = r[k]
        if "roofline" in keep:
            keep["roofline"] = {k: v for k, v in keep["roofline"].items()
                                if k not in ("isolated_launch_ms", "timing")}
        keep["wall_s"] = round(time.perf_counter() - t1, 2)
        out[cfg] = keep
    torch.cuda.empty_cache()
    out["wall_s"] = round(time.perf_counter() - t0, 2)
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    rank, world, device, dist = dist_setup(args)
    # Before any work: which GPU each rank drives; N ranks on fewer GPUs
    # fail the line here (outside a rehearsal).
    topology = gather_topology(local_topology(device), dist, os.environ.get("CIO_BENCH_REHEARSE") == "1")
    if args.config == "sha1":
        res = run_sha1(args, rank, world, device, dist)
    elif args.config == "e2e":
        res = run_e2e(args, rank, world, device, dist)
    elif args.config == "perf":
        res = run_perf(args, rank, world, device, dist)
    elif args.config == "verify":
        res = run_verify(args, rank, world, device, dist)
    elif args.config == "multi":
        multi = multi_device_host_leg(args, rank, world, device, dist)
        res = {"metric": "single-process all-devices host-memory CRC32 GB/s (cio_crc32_batch_host_multi)",
               "value": multi["host_batch_multi"]["GBps"] if multi else None, "unit": "GB/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "u8", "data": "synthetic, pageable host memory",
               "config": {"workload": "weak cfg2 job of N GPUs from one process, devices 0..N-1"},
               "multi_device_host": multi}
    else:
        res = run_crc(args, rank, world, device, dist)
        if args.config == "cfg2" and not args.no_extra:
            # The host-memory legs (e2e, verify, perf) run before the legs
            # that allocate and free tens of GB of HBM (cfg4: 34 GB, cfg3:
            # 40 GB): the driver clears freed VRAM in the background on the
            # SDMA engines the H2D copies use, which slows host batches by
            # ~11% for ~1 s after such a free (profiles/r04/e2e_vram_free/README.md).
            host_legs = other_configs(args, rank, world, device, dist, only=("e2e", "verify", "perf"))
            multi = multi_device_host_leg(args, rank, world, device, dist)
            if multi is not None:
                res["multi_device_host"] = multi
            res["other_chunk_sizes"] = other_chunk_sizes(args, rank, world, device, dist)
            dev_legs = other_configs(args, rank, world, device, dist, only=("cfg3", "sha1"))
            wall = host_legs.pop("wall_s") + dev_legs.pop("wall_s")
            res["other_configs"] = {**dev_legs, **host_legs, "wall_s": round(wall, 2),
                                    "order": "run order: e2e, verify, perf (host-memory legs, before any "
                                             "multi-GB HBM free), then other_chunk_sizes, cfg3, sha1"}
            res["diagnostic_batches"] = diagnostic_batches(device)
    res["topology"] = topology
    if world > 1:
        res.setdefault("per_gpu", {}).update(
            {k: topology[k] for k in ("device_index", "pci_bus_id", "numa_node")})
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
