#!/bin/bash
# Round-5 GPU session y: anti-camping grid tests, then the whole GPU suite.
set -u
O=gpurun_out/${1:-r05y}
mkdir -p $O
export TMPDIR=/tmp
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_crc.py -k anticamp -x -v -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest_anticamp.txt 2>&1; step $? anticamp
grep -E "passed|failed" $O/pytest_anticamp.txt | tail -1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1; step $? pytest
tail -1 $O/pytest_gpu.txt
echo all-done
