#!/bin/bash
# SHA-1 diagnostics: round wave exec mask (half / full) and grid size.
set -u
OUT=gpurun_out/r03j; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
M=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 200 python tools/sha1_ab.py --diag --libs $M,$A/sha1_c64half.so,$A/sha1_c32s1.so,$A/sha1_c32s1full.so --rounds 5 --iters 10 > $OUT/ab_sha1_exec.txt 2>&1 || exit $?
timeout -k 10 200 python tools/sha1_ab.py --chunks 512 --libs $M,$A/sha1_c32s1.so --rounds 5 --iters 10 > $OUT/ab_sha1_512.txt 2>&1 || exit $?
timeout -k 10 200 python tools/sha1_ab.py --chunks 256 --libs $M,$A/sha1_c32s1.so --rounds 5 --iters 10 > $OUT/ab_sha1_256.txt 2>&1 || exit $?
grep -h "ms/call" $OUT/ab_sha1_exec.txt $OUT/ab_sha1_512.txt $OUT/ab_sha1_256.txt
