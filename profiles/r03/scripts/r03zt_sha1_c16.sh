#!/bin/bash
# SHA-1 A/B on the anchored kernel: 16 chunks per workgroup (CIO_SHA1_CHAINS=16
# against the product's 32 with 1), interleaved.
set -u
OUT=gpurun_out/${1:-r03zt}; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
timeout -k 10 300 python tools/sha1_ab.py --libs chunkio_amd/lib/libchunkio_amd.so,$A/sha1_c16.so --rounds 5 --iters 10 > $OUT/ab_sha1_c16.txt 2>&1 || { tail -20 $OUT/ab_sha1_c16.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_sha1_c16.txt | tail -5
