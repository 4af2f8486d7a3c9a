#!/bin/bash
# Round-5 GPU session (tag $1, default r05k): the GPU suite with the learned split route, the split
# probe (with and without NUMA binding), and the default line.
set -u
O=gpurun_out/${1:-r05k}
mkdir -p $O
export TMPDIR=/tmp
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1; step $? pytest
tail -2 $O/pytest_gpu.txt
CIOA_ROUTE_DEBUG=1 timeout -k 10 400 python -u tools/split_probe.py 3 > $O/split_probe.txt 2> $O/split_probe.err; step $? probe
SPLIT_PROBE_BIND=1 CIOA_ROUTE_DEBUG=1 timeout -k 10 400 python -u tools/split_probe.py 3 > $O/split_probe_bind.txt 2> $O/split_probe_bind.err; step $? probe_bind
tail -12 $O/split_probe.txt; tail -12 $O/split_probe_bind.txt
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err; step $? default
echo all-done
