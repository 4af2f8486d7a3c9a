#!/bin/bash
# SHA-1 A/B: lanes 32-63 of the round wave (duplicate chains) skip the row reads
# (-DCIO_SHA1_HALF_READS) against the product kernel, interleaved.
set -u
OUT=gpurun_out/${1:-r03zo}; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
timeout -k 10 300 python tools/sha1_ab.py --libs chunkio_amd/lib/libchunkio_amd.so,$A/sha1_half_reads.so --rounds 5 --iters 10 > $OUT/ab_sha1_half_reads.txt 2>&1 || { tail -20 $OUT/ab_sha1_half_reads.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_sha1_half_reads.txt | tail -4
