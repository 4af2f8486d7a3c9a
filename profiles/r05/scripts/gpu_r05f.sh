#!/bin/bash
# Round-5 GPU session f: the GPU suite with the split route, and the default line.
set -u
O=gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1; step $? pytest
tail -2 $O/pytest_gpu.txt
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err; step $? default
echo all-done
