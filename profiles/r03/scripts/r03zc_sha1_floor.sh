#!/bin/bash
# SHA-1 wave kernel (A/B build) floors: rounds only (no scalar loads, no waits),
# loads without waits, and the real kernel, on the whole cfg5 batch (every SIMD
# busy) and on a quarter of it (64 CUs busy): is the floor the chip's clock
# under whole-chip load or the loads' issue?  Timing only (--diag).
set -u
OUT=gpurun_out/${1:-r03zc}; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
L=$A/sha1_old.so,$A/sha1_wave.so,$A/sha1_wave_nowait.so,$A/sha1_wave_noload.so
timeout -k 10 300 python tools/sha1_ab.py --diag --libs $L --rounds 3 --iters 5 > $OUT/sha1_floor_1024.txt 2>&1 || { tail -20 $OUT/sha1_floor_1024.txt; exit 1; }
grep -h "ms/call" $OUT/sha1_floor_1024.txt
timeout -k 10 300 python tools/sha1_ab.py --diag --chunks 256 --libs $L --rounds 3 --iters 5 > $OUT/sha1_floor_256.txt 2>&1 || { tail -20 $OUT/sha1_floor_256.txt; exit 1; }
grep -h "ms/call" $OUT/sha1_floor_256.txt
