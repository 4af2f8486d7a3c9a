#!/bin/bash
# Round-5 GPU session g: sanitizers on the GPU route, now also the split route.
set -u
O=gpurun_out/${1:-r05g}
mkdir -p $O
export TMPDIR=/tmp
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
timeout -k 10 500 bash tools/asan_check.sh gpu > $O/asan_gpu.txt 2>&1; step $? asan-gpu
timeout -k 10 500 bash tools/asan_check.sh tsan-gpu > $O/tsan_gpu.txt 2>&1; step $? tsan-gpu
echo all-done
