#!/bin/bash
# SHA-1 final kernel: GPU tests, then A/B against the round-2/3 kernel (ab/sha1_old.so).
set -u
OUT=gpurun_out/r03j; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
M=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sha1.py > $OUT/pytest_sha1.txt 2>&1 || { tail -30 $OUT/pytest_sha1.txt; exit 1; }
tail -2 $OUT/pytest_sha1.txt
timeout -k 10 300 python tools/sha1_ab.py --libs $A/sha1_old.so,$M --rounds 7 --iters 10 > $OUT/ab_sha1_final.txt 2>&1 || exit $?
grep -h "ms/call\|digests" $OUT/ab_sha1_final.txt
