#!/bin/bash
# SHA-1 lane-shared rows (DPP): SHA-1 GPU tests on the default build, then
# interleaved A/Bs against the previous kernel (ab/sha1_old.so): the DPP add
# 0/1/2 rounds ahead of its use, 4 lanes per chunk, and a diagnostic build
# with the DPP read replaced by a plain add (wrong digests: timing only).
set -u
OUT=gpurun_out/${1:-r03p}; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
M=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sha1.py > $OUT/pytest_sha1.txt 2>&1 || { tail -30 $OUT/pytest_sha1.txt; exit 1; }
tail -2 $OUT/pytest_sha1.txt
timeout -k 10 300 python tools/sha1_ab.py --libs $A/sha1_old.so,$M,${VARS:-$A/sha1_l2a0.so,$A/sha1_l2a1.so,$A/sha1_l4.so} --rounds 5 --iters 10 > $OUT/ab_sha1_lanes.txt 2>&1 || { tail -20 $OUT/ab_sha1_lanes.txt; exit 1; }
grep -h "ms/call\|digests" $OUT/ab_sha1_lanes.txt
if [ -n "${DIAG:-$A/sha1_l2nodpp.so}" ]; then
  timeout -k 10 300 python tools/sha1_ab.py --diag --libs $A/sha1_old.so,$M,${DIAG:-$A/sha1_l2nodpp.so} --rounds 5 --iters 10 > $OUT/ab_sha1_diag.txt 2>&1 || { tail -20 $OUT/ab_sha1_diag.txt; exit 1; }
  grep -h "ms/call" $OUT/ab_sha1_diag.txt
fi
