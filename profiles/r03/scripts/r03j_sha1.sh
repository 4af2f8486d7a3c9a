#!/bin/bash
# SHA-1: chunks per workgroup (64/32/16), schedule waves, group size; interleaved A/B.
set -u
OUT=gpurun_out/r03j; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
L=chunkio_amd/lib/libchunkio_amd.so,$A/sha1_c32s2.so,$A/sha1_c32s1.so,$A/sha1_c16s1.so,$A/sha1_c32s1g2.so,$A/sha1_c16s1g8.so,$A/sha1_c32s1g8.so,$A/sha1_c32s2g8.so
timeout -k 10 400 python tools/sha1_ab.py --libs $L --rounds 5 --iters 10 > $OUT/ab_sha1_chains.txt 2>&1 || exit $?
cat $OUT/ab_sha1_chains.txt | tail -12
