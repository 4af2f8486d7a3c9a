#!/bin/bash
# SHA-1 A/B: 4 chunks per workgroup with 16 blocks per barrier (A/B build, its
# default geometry forced with CIO_SHA1_CHUNKS_PER_WG=32) against the product
# (8/8 for this batch), separate processes alternated.
set -u
OUT=gpurun_out/${1:-r03zw}; mkdir -p $OUT; export TMPDIR=/tmp
: > $OUT/ab_sha1_c4.txt
for pass in 1 2 3; do
  timeout -k 10 200 python tools/sha1_ab.py --libs chunkio_amd/lib/libchunkio_amd.so --rounds 2 --iters 10 2>&1 | grep "ms/call" | sed "s/^/pass $pass /" >> $OUT/ab_sha1_c4.txt || exit 1
  CIO_SHA1_CHUNKS_PER_WG=32 timeout -k 10 200 python tools/sha1_ab.py --libs chunkio_amd/lib/ab/sha1_c4g16.so --rounds 2 --iters 10 2>&1 | grep -E "ms/call|digests" | sed "s/^/pass $pass /" >> $OUT/ab_sha1_c4.txt || exit 1
done
cat $OUT/ab_sha1_c4.txt
