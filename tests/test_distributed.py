"""Multi-process sharding (world_size 2, gloo, CPU): chunk i -> rank i mod 2,
no collective on the data path, results gathered by index.  Each rank CRCs
its shard with the library's host crc_update (the CPU drop-in), which is all
a CPU rank can run; the GPU ranks run the same shard logic in bench.py."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from chunkio_amd import shard
from chunkio_amd import workloads as wl


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, seed, q):
    import torch.distributed as dist
    import chunkio_amd as cio
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lens = (np.arange(n) * 977 % 20000).astype(np.uint64)
        ids = shard.shard_ids(n, rank, world)
        local = np.asarray([cio.crc_update(0xFFFFFFFF, wl.gen_chunk(seed, int(i), int(lens[i])))
                            for i in ids], dtype=np.uint32)
        full = shard.gather_results(local, n)
        only0 = shard.gather_results(local, n, dst=0)
        if rank == 0:
            q.put((full, only0))
        else:
            assert only0 is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_shard_ids_partition():
    for n in (0, 1, 7, 1024, 8192):
        for world in (1, 2, 3, 8):
            ids = np.concatenate([shard.shard_ids(n, r, world) for r in range(world)])
            assert sorted(ids.tolist()) == list(range(n))
    with pytest.raises(ValueError):
        shard.shard_ids(10, 2, 2)


def test_assemble_roundtrip():
    n, world = 37, 3
    vals = np.arange(n, dtype=np.uint32) * 7
    parts = [vals[shard.shard_ids(n, r, world)] for r in range(world)]
    np.testing.assert_array_equal(shard.assemble(n, world, parts), vals)


def test_gloo_world2_sharded_crc():
    from oracle import pyoracle as po
    n, seed, world = 101, 0xC1000004, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, only0 = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    lens = (np.arange(n) * 977 % 20000).astype(np.uint64)
    want = np.asarray([po.crc_update(0xFFFFFFFF, wl.gen_chunk(seed, i, int(lens[i]))) for i in range(n)],
                      dtype=np.uint32)
    np.testing.assert_array_equal(full, want)
    np.testing.assert_array_equal(only0, want)


def test_bench_geometry_shards_cover_job():
    import bench
    for cfg in ("cfg2", "cfg4"):
        seen = []
        for r in range(4):
            lens, ids, seed, desc, scaling = bench.geometry(cfg, r, 4)
            seen.append(ids)
            assert len(lens) == len(ids)
        allids = np.sort(np.concatenate(seen))
        if cfg == "cfg4":      # strong scaling: the 8192-chunk job split four ways
            assert allids.tolist() == list(range(wl.CFG4_N))
        else:                  # weak scaling: 1024 chunks per GPU
            assert allids.tolist() == list(range(4 * wl.CFG2_N))


def _gather_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        got = bench.gather_over_ranks(10.0 + rank, dist, "cpu")
        mx = bench.max_over_ranks(float(rank), dist, "cpu")
        if rank == 0:
            q.put((got, mx))
    finally:
        dist.destroy_process_group()


def test_bench_rank_reductions_gloo_world2():
    """bench.py's max-over-ranks and per-GPU gather on the gloo backend."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, mx = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == [10.0, 11.0]
    assert mx == 1.0


def test_bench_gpus_n_spawns_ranks_or_refuses(tmp_path):
    """`python bench.py --gpus N` with no launcher environment starts N rank
    processes itself (bench.spawn_ranks) and refuses, non-zero, when fewer
    than N GPUs are visible -- here, on a CPU host, with none visible."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2, r.stderr
    assert "--gpus 2 but only 0 GPU(s) visible" in r.stderr
    assert r.stdout == ""


def test_bench_spawn_parent_counts_gpus_without_torch():
    """The spawn parent counts GPUs from sysfs and never imports torch (so it
    cannot initialise the GPU before its children start); here, no GPU."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); import bench; n, how = bench.visible_gpus(); "
            "print(n, how.split('+')[0], 'torch' in sys.modules)" % root)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    n, how, imported = r.stdout.split()
    assert (n, how, imported) == ("0", "kfd-sysfs", "False")


def test_bench_traffic_scales_to_a_shards_launch():
    """roofline.traffic at N > 1: a strong-scaled cfg4 shard launches 1/N of the
    bytes the committed N = 1 PMC pass profiled, so the bench applies that
    pass's traffic/algorithmic ratio instead of its absolute bytes."""
    import json
    import bench
    with open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                           "profiles", "pmc_cfg4.json")) as f:
        d = json.load(f)
    full = d["algorithmic_bytes_per_launch"]
    assert bench.load_pmc_traffic("cfg4", full) == d["hbm_bytes_per_launch"]
    for world in (2, 4, 8):
        got = bench.load_pmc_traffic("cfg4", full // world)
        assert got == round(d["traffic_over_algorithmic"] * (full // world))
    assert bench.load_pmc_traffic("no_such_config", 1) is None


def test_gloo_init_keeps_stdout_clean():
    """Two ranks through bench.init_gloo_quiet: gloo's connection messages
    land on stderr, so rank 0's stdout is exactly what bench.py prints (the
    driver reads one JSON line there)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, json; sys.path.insert(0, %r); import bench; d = bench.init_gloo_quiet(); "
            "print(json.dumps({'rank': d.get_rank()})); d.destroy_process_group()" % root)
    port = str(29500 + os.getpid() % 1000)
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-2000:] for o in outs]
    for r, (out, _) in enumerate(outs):
        assert out.splitlines() == ['{"rank": %d}' % r], out


def _spawn_bench(extra_env, gpus=2):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(CIO_BENCH_REHEARSE="1", **extra_env)
    return subprocess.Popen([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(gpus),
                             "--steps", "1", "--warmup", "0"], env=env,
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)


def _rank_pids(stderr):
    import re
    return [int(m) for m in re.findall(r"bench\.py: rank \d+ pid (\d+)", stderr)]


def _gone(pid):
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return True
    # a zombie not yet reaped by init still answers kill(0); check its state
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split(")")[-1].split()[0] == "Z"
    except OSError:
        return True


@pytest.mark.parametrize("fail_at", ["barrier", "init"])
def test_bench_spawn_fails_fast_when_a_rank_dies(fail_at):
    """`bench.py --gpus 2` with rank 1 forced to exit 1 (after the gloo
    rendezvous, with rank 0 waiting in a barrier; or before it, with rank 0
    waiting in the rendezvous): the launcher sees the failure, stops rank 0
    and returns non-zero within seconds -- not after gloo's timeout -- and
    leaves no rank process behind."""
    import time
    t0 = time.monotonic()
    p = _spawn_bench({"CIO_BENCH_FAIL_RANK": "1", "CIO_BENCH_FAIL_AT": fail_at})
    out, err = p.communicate(timeout=120)
    took = time.monotonic() - t0
    assert p.returncode not in (0, None), err[-2000:]
    assert took < 60, took
    assert out == ""
    pids = _rank_pids(err)
    assert len(pids) == 2, err[-2000:]
    assert "rank 1 exited with status 1" in err or "exited with status" in err, err[-2000:]
    time.sleep(0.5)
    assert all(_gone(pid) for pid in pids), pids


def test_bench_spawn_forwards_sigterm_to_ranks():
    """A hung rank (rank 1 never reaches the barrier): SIGTERM to the launcher
    (a driver's time limit) stops every rank before the launcher exits."""
    import signal
    import time
    p = _spawn_bench({"CIO_BENCH_FAIL_RANK": "1", "CIO_BENCH_FAIL_AT": "hang",
                      "CIO_BENCH_PG_TIMEOUT_S": "600"})
    # wait until both ranks are up (their pids are printed as they start)
    import selectors
    sel = selectors.DefaultSelector()
    sel.register(p.stderr, selectors.EVENT_READ)
    buf = ""
    t0 = time.monotonic()
    while len(_rank_pids(buf)) < 2 and time.monotonic() - t0 < 60:
        if sel.select(timeout=1):
            line = p.stderr.readline()
            if not line:
                break
            buf += line
    pids = _rank_pids(buf)
    assert len(pids) == 2, buf
    time.sleep(3)                        # ranks importing torch / in the rendezvous
    p.send_signal(signal.SIGTERM)
    p.communicate(timeout=60)
    assert p.returncode == 128 + signal.SIGTERM
    time.sleep(0.5)
    assert all(_gone(pid) for pid in pids), pids


def test_bench_pg_timeout_bounds_a_barrier_without_the_launcher():
    """Ranks started by another launcher (torch.distributed.run): a barrier on a
    dead peer ends with an error within the bounded gloo timeout, not 30 min."""
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); import bench, os; d = bench.init_gloo_quiet(); "
            "r = d.get_rank()\n"
            "if r == 1: os._exit(1)\n"
            "d.barrier()" % root)
    port = str(_free_port())
    procs = []
    t0 = time.monotonic()
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, CIO_BENCH_PG_TIMEOUT_S="10")
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    for p in procs:
        p.communicate(timeout=120)
    assert procs[1].returncode == 1
    assert procs[0].returncode != 0
    assert time.monotonic() - t0 < 60


def _job_digest_worker(rank, world, port, want, want_rows, q):
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 37
        job = (np.arange(n, dtype=np.uint64) * 0x9E3779B1 % (1 << 32)).astype(np.uint32)
        local = job[shard.shard_ids(n, rank, world)]
        ok = bench.job_digest_matches(local, n, want, dist)
        bad = local.copy()
        if rank == world - 1:
            bad[-1] ^= 1
        nok = bench.job_digest_matches(bad, n, want, dist)
        rows = np.random.default_rng(5).integers(0, 256, (n, 20), dtype=np.uint8)
        rok = bench.job_digest_matches(rows[shard.shard_ids(n, rank, world)], n, want_rows, dist)
        if rank == 0:
            q.put((ok, nok, rok))
        else:
            assert ok is None and nok is None and rok is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_job_digest_gathers_shards(world):
    """bench.py's full-job check at N > 1: every rank's round-robin shard
    (u32 CRCs, or 20-byte SHA-1 digests) gathered to rank 0 in job order; one
    flipped bit on the last rank fails it."""
    import hashlib
    import bench
    n = 37
    job = (np.arange(n, dtype=np.uint64) * 0x9E3779B1 % (1 << 32)).astype(np.uint32)
    want = hashlib.sha256(job.astype("<u4").tobytes()).hexdigest()
    assert bench.job_digest_matches(job, n, want, None) is True
    assert bench.job_digest_matches(job[:-1], n, want, None) is False
    rows = np.random.default_rng(5).integers(0, 256, (n, 20), dtype=np.uint8)
    want_rows = hashlib.sha256(rows.tobytes()).hexdigest()
    assert bench.job_digest_matches(rows, n, want_rows, None) is True
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_job_digest_worker, args=(r, world, port, want, want_rows, q))
             for r in range(world)]
    for p in procs:
        p.start()
    ok, nok, rok = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert ok is True and nok is False and rok is True


def _topology_worker(rank, world, port, rehearse, same_bus, q):
    import os
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        local = {"device_index": 0 if same_bus else rank, "numa_node": rank,
                 "pci_bus_id": "0000:05:00.0" if same_bus else f"0000:{5 + rank:02x}:00.0",
                 "host": "box", "pid": 100 + rank}
        try:
            out = bench.gather_topology(local, dist, rehearse)
            q.put((rank, "ok", out))
        except SystemExit as e:
            q.put((rank, "exit", str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("same_bus,rehearse,want", [(False, False, "ok"), (True, True, "ok"),
                                                     (True, False, "exit")])
def test_bench_topology_gather_gloo_world2(same_bus, rehearse, want):
    """bench.py records each rank's device index, PCI bus ID and NUMA node
    (gloo all_gather_object), and two ranks on one GPU fail the line on every
    rank unless CIO_BENCH_REHEARSE asked for exactly that."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_topology_worker, args=(r, 2, port, rehearse, same_bus, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert [g[1] for g in got] == [want, want]
    if want == "ok":
        topo = got[0][2]
        assert topo == got[1][2]
        assert topo["numa_node"] == [0, 1] and topo["ranks"] == 2
        assert topo["distinct_gpus"] == (1 if same_bus else 2)
        assert topo["pci_bus_id"] == (["0000:05:00.0"] * 2 if same_bus else ["0000:05:00.0", "0000:06:00.0"])
    else:
        assert "share a GPU" in got[0][2]


def test_bench_cpu_baselines_at_n2():
    """The CPU legs bench.py puts beside every line, as rank 0 runs them at
    N = 2: the reference crc32.c (1 thread + the per-GPU share) over a CRC
    batch, and OpenSSL SHA-1 over a SHA-1 batch, each bit-exact against the
    expected outputs (the oracle / hashlib stand in for the GPU's here)."""
    import hashlib
    import bench
    from oracle import pyoracle as po
    rng = np.random.default_rng(4)
    lens = np.full(64, 4096, dtype=np.uint64)
    offs = wl.packed_offsets(lens, align=16)
    host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    want = po.crc_batch(host, offs, lens)
    r = bench.cpu_baseline(host, offs, lens, want, world=2, reps=4, perf=False)
    assert r["cores"] == 1 and r["kind"] in ("reference", "port") and r["bit_exact_vs_gpu"]
    assert r["multi_thread"]["threads"] == bench.cpu_share(2) or "multi_thread" not in r
    assert r["value"] > 0
    dig = np.frombuffer(b"".join(hashlib.sha1(host[int(o):int(o + n)]).digest() for o, n in zip(offs, lens)),
                        np.uint8).reshape(-1, 20)
    s = bench.sha1_cpu_baseline(host, offs, lens, dig, world=2)
    assert s["cores"] == 1 and s["bit_exact_vs_gpu"] and s["value"] > 0 and s["shard"].startswith("rank 0")
    if bench.cpu_share(2) > 1:
        assert s["multi_thread"]["bit_exact_vs_gpu"] and s["multi_thread"]["threads"] == bench.cpu_share(2)
    bad = dig.copy()
    bad[3, 0] ^= 1
    assert not bench.sha1_cpu_baseline(host, offs, lens, bad, world=2)["bit_exact_vs_gpu"]


def _multi_leg_worker(rank, world, port, q):
    import os
    import time
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = []

        def runner(args, w, device):
            calls.append(w)
            time.sleep(0.5)                 # the others must wait for rank 0 here
            return {"devices": bench.multi_device_list(w, 1, True)[0]}
        t0 = time.perf_counter()
        res = bench.multi_device_host_leg(None, rank, world, "cpu", dist, runner=runner)
        q.put((rank, res, calls, time.perf_counter() - t0))
    finally:
        dist.destroy_process_group()


def test_bench_multi_device_leg_rank0_alone_gloo_world2():
    """bench.py's all-devices host leg at world size 2 on gloo: rank 0 alone
    runs the single-process multi-device calls (a stub here: no GPU on this
    side) while rank 1 waits at the leg's barriers, and only rank 0's line
    carries the result; the device list is 0..N-1, or the visible GPUs
    round-robin in a rehearsal, and refused otherwise."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_multi_leg_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(2):
        rank, res, calls, dt = q.get(timeout=120)
        out[rank] = (res, calls, dt)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert out[0][1] == [2] and out[1][1] == []
    assert out[0][0]["devices"] == [0, 0] and "wall_s" in out[0][0]
    assert out[1][0] is None
    assert out[1][2] >= 0.45                # rank 1 was held until rank 0 finished
    import bench
    assert bench.multi_device_list(8, 8, False) == (list(range(8)), False)
    assert bench.multi_device_list(2, 1, True) == ([0, 0], True)
    assert bench.multi_device_list(4, 2, True) == ([0, 1, 0, 1], True)
    assert bench.multi_device_list(2, 1, False) == (None, True)
    assert bench.multi_device_list(1, 1, False) == ([0], False)
