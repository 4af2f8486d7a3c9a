#!/bin/bash
# SHA-1 time breakdown: no schedule work / no LDS row reads / no rounds (diagnostic builds).
set -u
OUT=gpurun_out/r03j; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
M=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 300 python tools/sha1_ab.py --diag --libs $M,$A/sha1_d_nosched.so,$A/sha1_d_noread.so,$A/sha1_d_norounds.so,$A/sha1_d_nosched_noread.so,$A/sha1_c32s1full.so --rounds 5 --iters 10 > $OUT/ab_sha1_breakdown.txt 2>&1 || exit $?
grep -h "ms/call" $OUT/ab_sha1_breakdown.txt
