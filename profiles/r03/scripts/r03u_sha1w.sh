#!/bin/bash
# SHA-1 wave kernel with 40-word segments and cross-pass prefetch: SHA-1 GPU tests, A/B against the
# 32-chunk kernel (ab/sha1_old.so), and the no-wait diagnostic (timing only).
set -u
OUT=gpurun_out/${1:-r03u}; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
M=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sha1.py > $OUT/pytest_sha1.txt 2>&1 || { tail -40 $OUT/pytest_sha1.txt; exit 1; }
tail -2 $OUT/pytest_sha1.txt
timeout -k 10 300 python tools/sha1_ab.py --libs $A/sha1_old.so,$M --rounds 5 --iters 10 > $OUT/ab_sha1_wave40.txt 2>&1 || { tail -20 $OUT/ab_sha1_wave40.txt; exit 1; }
grep -h "ms/call\|digests" $OUT/ab_sha1_wave40.txt
timeout -k 10 300 python tools/sha1_ab.py --diag --libs $M,$A/sha1_wv40_nowait.so --rounds 3 --iters 5 > $OUT/ab_sha1_wave40_diag.txt 2>&1 || { tail -20 $OUT/ab_sha1_wave40_diag.txt; exit 1; }
grep -h "ms/call" $OUT/ab_sha1_wave40_diag.txt
