#!/bin/bash
# Round-5 GPU session z: the >4 GiB chunk test, then the whole GPU suite.
set -u
O=gpurun_out/${1:-r05z}
mkdir -p $O
export TMPDIR=/tmp
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_crc.py -k "4gib" -x -v -p no:cacheprovider \
    --timeout 120 --timeout-method thread --durations=5 > $O/pytest_4gib.txt 2>&1; step $? t4gib
grep -E "passed|failed|s call" $O/pytest_4gib.txt | tail -4
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1; step $? pytest
tail -1 $O/pytest_gpu.txt
echo all-done
