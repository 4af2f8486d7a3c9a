#!/bin/bash
# With the L64 layout: issue-ahead (two slots) against one slot, by shape.
set -u
OUT=gpurun_out/r03h; mkdir -p $OUT; export TMPDIR=/tmp
L=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 400 python tools/ab_lib.py --libs $L,$L --env 'CIO_GPU_AHEAD=0|CIO_GPU_AHEAD=1' --cfg cfg2,mid,big --iters 200 --rounds 4 > $OUT/ab_ahead_l64.txt 2>&1 || exit $?
tail -1 $OUT/ab_ahead_l64.txt
