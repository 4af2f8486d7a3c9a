#!/bin/bash
# SHA-1 wave kernel diagnostics (timing only, --diag): no waits for the
# scalar loads (pure issue rate), scalar-cache hits allowed (no glc), and the
# default kernel on a quarter of the batch (256 chunks: 64 workgroups).
set -u
OUT=gpurun_out/${1:-r03s}; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
M=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 300 python tools/sha1_ab.py --diag --libs $A/sha1_old.so,$M,$A/sha1_wv_nowait.so,$A/sha1_wv_noglc.so --rounds 3 --iters 5 > $OUT/ab_sha1_wave_diag.txt 2>&1 || { tail -20 $OUT/ab_sha1_wave_diag.txt; exit 1; }
grep -h "ms/call" $OUT/ab_sha1_wave_diag.txt
timeout -k 10 300 python tools/sha1_ab.py --libs $A/sha1_old.so,$M --chunks 256 --rounds 3 --iters 5 > $OUT/ab_sha1_wave_256.txt 2>&1 || { tail -20 $OUT/ab_sha1_wave_256.txt; exit 1; }
grep -h "ms/call" $OUT/ab_sha1_wave_256.txt
