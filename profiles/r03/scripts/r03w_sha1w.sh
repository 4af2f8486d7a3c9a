#!/bin/bash
# SHA-1 wave kernel with the rounds on fewer lanes (exec = 1 lane / 32 lanes):
# power per instruction vs the chip's clock with every SIMD busy.
set -u
OUT=gpurun_out/${1:-r03w}; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
M=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 300 python tools/sha1_ab.py --libs $A/sha1_old.so,$M,$A/sha1_wv_e1.so,$A/sha1_wv_e32.so --rounds 5 --iters 10 > $OUT/ab_sha1_wave_exec.txt 2>&1 || { tail -20 $OUT/ab_sha1_wave_exec.txt; exit 1; }
grep -h "ms/call\|digests" $OUT/ab_sha1_wave_exec.txt
