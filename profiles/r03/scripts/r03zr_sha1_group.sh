#!/bin/bash
# SHA-1 A/B on the anchored kernel: blocks handed over per barrier (CIO_SHA1_GROUP
# 2 and 8 against the product's 4), interleaved.
set -u
OUT=gpurun_out/${1:-r03zr}; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
timeout -k 10 300 python tools/sha1_ab.py --libs chunkio_amd/lib/libchunkio_amd.so,$A/sha1_group2.so,$A/sha1_group8.so --rounds 5 --iters 10 > $OUT/ab_sha1_group.txt 2>&1 || { tail -20 $OUT/ab_sha1_group.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_sha1_group.txt | tail -5
