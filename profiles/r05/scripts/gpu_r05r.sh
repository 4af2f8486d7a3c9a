#!/bin/bash
# Round-5 GPU session r: HBM channel camping vs per-wave range size -- the
# read-only stream at w steps per wave on 256 and 255 workgroups, and the CRC
# kernels with one workgroup fewer (CIO_GPU_GRID) on power-of-two batches.
set -u
O=gpurun_out/r05r
mkdir -p $O
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
timeout -k 10 500 python tools/rs_size_probe.py 16,17,25,32,64,128,256,512 256,255,252 > $O/rs_size_grid.txt 2>&1; step $? rs
tail -10 $O/rs_size_grid.txt
timeout -k 10 600 python tools/ab_lib.py --libs chunkio_amd/lib/libchunkio_amd.so,chunkio_amd/lib/libchunkio_amd.so --env "|CIO_GPU_GRID=255" --cfg k4x65536,k4x131072,big,cfg2,cfg4k,mid \
    --iters 30 --rounds 3 > $O/ab_grid255.txt 2>&1; step $? ab255
tail -1 $O/ab_grid255.txt
timeout -k 10 600 python tools/ab_lib.py --libs chunkio_amd/lib/libchunkio_amd.so,chunkio_amd/lib/libchunkio_amd.so --env "|CIO_GPU_GRID=1020" --cfg cfg4 \
    --iters 6 --rounds 3 > $O/ab_grid1020.txt 2>&1; step $? ab1020
tail -1 $O/ab_grid1020.txt
echo all-done
