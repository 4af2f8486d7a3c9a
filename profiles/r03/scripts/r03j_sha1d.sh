#!/bin/bash
# SHA-1: block-pipelined round wave (next block's rows read during this block's rounds).
set -u
OUT=gpurun_out/r03j; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
M=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 300 python tools/sha1_ab.py --libs $M,$A/sha1_pipe.so,$A/sha1_pipe_g2.so,$A/sha1_pipe_c32s1.so,$A/sha1_pipe_c32s1g8.so,$A/sha1_pipe_c32s2g8.so,$A/sha1_c32s1full.so --rounds 5 --iters 10 > $OUT/ab_sha1_pipe.txt 2>&1 || exit $?
grep -h "ms/call\|digests" $OUT/ab_sha1_pipe.txt
