#!/bin/bash
# Round-5 GPU session u: anti-camping range cap (CIO_GPU_ANTICAMP_MAX) and
# the issue-ahead kernel on a reduced grid.
set -u
O=gpurun_out/${1:-r05u}
mkdir -p $O
export TMPDIR=/tmp
L=chunkio_amd/lib/libchunkio_amd.so
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
# stream kernel: 64 KiB chunks -> 16/32/64/128/256 steps per wave; small kernel 128/256 chunks per wave
timeout -k 10 500 python tools/ab_lib.py --libs $L,$L,$L --env "CIO_GPU_ANTICAMP=0||CIO_GPU_ANTICAMP_MAX=1023" \
    --cfg c64kx4096,c64kx8192,c64kx16384,c64kx32768,c64kx65536,big,k4x524288,k4x1048576,mid --iters 20 --rounds 3 > $O/ab_cap.txt 2>&1; step $? ab_cap
tail -1 $O/ab_cap.txt
timeout -k 10 300 python tools/ab_lib.py --libs $L,$L --env "|CIO_GPU_AHEAD=1" \
    --cfg c64kx16384,c64kx8192,k4x262144 --iters 30 --rounds 4 > $O/ab_ahead.txt 2>&1; step $? ab_ahead
tail -1 $O/ab_ahead.txt
echo all-done
