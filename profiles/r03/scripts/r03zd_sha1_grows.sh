#!/bin/bash
# A/B: the 32-chunk SHA-1 kernel with its K + W rows handed over through a
# per-workgroup ring in global memory (vector loads in the round wave) instead
# of LDS (-DCIO_SHA1_GLOBAL_ROWS); digests compared across builds + hashlib.
set -u
OUT=gpurun_out/${1:-r03zd}; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
M=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 300 python tools/sha1_ab.py --libs $M,$A/sha1_grows.so,$M,$A/sha1_grows.so --rounds 4 --iters 10 > $OUT/ab_sha1_grows.txt 2>&1 || { tail -20 $OUT/ab_sha1_grows.txt; exit 1; }
grep -h "ms/call\|digests" $OUT/ab_sha1_grows.txt
