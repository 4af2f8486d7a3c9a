#!/bin/bash
# SHA-1 A/B on the anchored kernel: chunks per workgroup (32 product, 16, 16 with
# 8 blocks per barrier, 8 with 8 blocks per barrier), interleaved.
set -u
OUT=gpurun_out/${1:-r03zu}; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
timeout -k 10 300 python tools/sha1_ab.py --libs chunkio_amd/lib/libchunkio_amd.so,$A/sha1_c16.so,$A/sha1_c16g8.so,$A/sha1_c8g8.so --rounds 5 --iters 10 > $OUT/ab_sha1_chains.txt 2>&1 || { tail -20 $OUT/ab_sha1_chains.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_sha1_chains.txt | tail -6
