#!/usr/bin/env python3
"""Time the reference binary `tools/cio -p tests/data/400kb.txt` (with and
without -k) against oracle/cio_perf_port.c, interleaved, in one container
(the port must be within noise of the binary).

The binary is the one tools/ref_dropin_ctest.sh builds from a /tmp copy of
the reference ($WORK/stock/build/tools/cio: unmodified sources, its own
deps/crc32).  The port runs twice: bound to the reference crc_update
(oracle/_ref, kind "reference") and to the oracle restatement ("port").
All three do 1000 files x 5 writes of 400 KB into /tmp and count the same
2,048,000,000 bytes; rates are bytes / elapsed as tools/cio.c:437-462 prints.

Baseline / harness infrastructure only; not part of the product or of any
GPU run.  Usage: python tools/ref_perf_timing.py [--reps 5] [--cio PATH]
"""
import argparse
import ctypes
import os
import re
import shutil
import statistics
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pyoracle as po  # noqa: E402

DATA = os.path.join(ROOT, "tests", "golden", "400kb.txt")


def run_binary(cio, checksum):
    cmd = [cio, "-p", DATA] + (["-k"] if checksum else [])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd="/tmp")
    if r.returncode != 0:
        raise RuntimeError(f"{cmd}: rc {r.returncode}\n{r.stderr}")
    m_rate = re.search(r"rate\s*:.*\(([\d.]+) bytes\)", r.stdout)
    m_bytes = re.search(r"bytes written\s*:.*\((\d+) bytes\)", r.stdout)
    m_crc = re.search(r"crc32 checksum : (\w+)", r.stdout)
    assert m_crc.group(1) == ("enabled" if checksum else "disabled"), r.stdout
    return float(m_rate.group(1)), int(m_bytes.group(1))


def settle():
    """Between legs: drop the binary's 2 GB of dirty output (it leaves its
    files in /tmp/cio-perf; the port deletes its own) and flush, so no leg
    pays for the previous leg's writeback."""
    shutil.rmtree("/tmp/cio-perf", ignore_errors=True)
    os.sync()


def run_port(lib, prefix, buf, checksum):
    d = tempfile.mkdtemp(prefix="cio_port_", dir="/tmp")
    try:
        nb = ctypes.c_uint64(0)
        secs = getattr(lib, prefix + "cio_perf_write")(d.encode(), buf.ctypes.data, buf.size, 1000, 5,
                                                     1 if checksum else 0, ctypes.byref(nb))
        if secs <= 0:
            raise RuntimeError("port failed")
        with open(os.path.join(d, "perf-test-0999.txt"), "rb") as f:
            head = f.read(10)
        return nb.value / secs, nb.value, head
    finally:
        shutil.rmtree(d, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cio", default="/tmp/cioa_ref_dropin/stock/build-release/tools/cio",
                    help="reference binary built -O3 (CMAKE_BUILD_TYPE=Release)")
    ap.add_argument("--cio-debug", default="/tmp/cioa_ref_dropin/stock/build/tools/cio",
                    help="reference binary as CIO_DEV builds it (Debug, -g, no -O)")
    a = ap.parse_args()
    for b in (a.cio, a.cio_debug):
        if not os.path.exists(b):
            sys.exit(f"{b} missing: run tools/ref_dropin_ctest.sh first")
    buf = np.fromfile(DATA, dtype=np.uint8)
    legs = {
        "binary -k": lambda: run_binary(a.cio, True),
        "binary(Debug) -k": lambda: run_binary(a.cio_debug, True),
        "port(ref crc) -k": lambda: run_port(po.ref(), "ref_", buf, True)[:2],
        "port(oracle crc) -k": lambda: run_port(po.oracle(), "oracle_", buf, True)[:2],
        "binary": lambda: run_binary(a.cio, False),
        "port(ref crc)": lambda: run_port(po.ref(), "ref_", buf, False)[:2],
    }
    # The port's files must be the binary's, byte for byte (3 files x 5 writes).
    subprocess.run([a.cio, "-p", DATA, "-k", "-e", "3"], check=True, capture_output=True, cwd="/tmp")
    d = tempfile.mkdtemp(prefix="cio_port_", dir="/tmp")
    nb = ctypes.c_uint64(0)
    po.ref().ref_cio_perf_write(d.encode(), buf.ctypes.data, buf.size, 3, 5, 1, ctypes.byref(nb))
    for i in range(3):
        name = f"perf-test-{i:04d}.txt"
        with open(os.path.join(d, name), "rb") as f1, open(os.path.join("/tmp/cio-perf/test-perf", name), "rb") as f2:
            x, y = f1.read(), f2.read()
        assert x == y, name
    print(f"port files == binary files (3 x {len(x)} B, header {x[:10].hex(' ')})")
    assert x[:10] == bytes.fromhex("c1 00 08 87 40 e7 00 00 00 00")
    shutil.rmtree(d)
    settle()
    names = list(legs)
    rates = {n: [] for n in names}
    for rep in range(a.reps):
        order = names if rep % 2 == 0 else names[::-1]
        for n in order:
            rate, nbytes = legs[n]()
            settle()
            assert nbytes == 2048000000, (n, nbytes)
            rates[n].append(rate)
        print(f"rep {rep}: " + "  ".join(f"{n} {rates[n][-1] / 1e6:.0f}" for n in names) + "  (MB/s)",
              flush=True)
    print(f"\n{os.cpu_count()} CPUs; 1000 files x 5 writes x 409600 B = 2,048,000,000 B per run; "
          f"{a.reps} interleaved reps (order reversed on odd reps; outputs deleted + sync "
          f"between legs); MB/s = 1e6 B/s")
    print(f"{'leg':22s} {'median':>8s} {'min':>8s} {'max':>8s}")
    for n in names:
        r = rates[n]
        print(f"{n:22s} {statistics.median(r) / 1e6:8.0f} {min(r) / 1e6:8.0f} {max(r) / 1e6:8.0f}")
    for pair in (("port(ref crc) -k", "binary -k"), ("binary(Debug) -k", "binary -k"), ("port(oracle crc) -k", "binary -k"),
                 ("port(ref crc)", "binary")):
        print(f"{pair[0]} / {pair[1]}: {statistics.median(rates[pair[0]]) / statistics.median(rates[pair[1]]):.3f}")


if __name__ == "__main__":
    main()
