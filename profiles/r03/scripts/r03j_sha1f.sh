#!/bin/bash
# SHA-1: pipelined round wave with the LDS row reads exec-masked to the workgroup's chunks.
set -u
OUT=gpurun_out/r03j; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
M=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 300 python tools/sha1_ab.py --libs $M,$A/sha1_pipe_c32s1.so,$A/sha1_pipe_c32m.so,$A/sha1_pipe.so --rounds 7 --iters 10 > $OUT/ab_sha1_masked_asm.txt 2>&1 || exit $?
grep -h "ms/call\|digests" $OUT/ab_sha1_masked_asm.txt
