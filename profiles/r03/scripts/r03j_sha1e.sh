#!/bin/bash
# SHA-1: cost of the hand-over barriers (diagnostic build without them) and the round probe.
set -u
OUT=gpurun_out/r03j; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
M=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 300 python tools/sha1_ab.py --diag --libs $M,$A/sha1_pipe_c32s1.so,$A/sha1_d_nobar.so,$A/sha1_d_nobar_noread.so,$A/sha1_d_nobar_nosched.so,$A/sha1_d_nobar_nosched_noread.so --rounds 5 --iters 10 > $OUT/ab_sha1_nobar2.txt 2>&1 || exit $?
grep -h "ms/call" $OUT/ab_sha1_nobar2.txt
