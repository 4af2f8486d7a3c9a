#!/bin/bash
# SHA-1 round wave with the chaining-value anchor (product build) against the
# same kernel without it (-DCIO_SHA1_NO_ANCHOR), interleaved; then the clock
# diagnostic of the anchored kernel, the SHA-1 GPU tests and the default bench.
set -u
OUT=gpurun_out/${1:-r03zl}; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
timeout -k 10 300 python tools/sha1_ab.py --libs $A/sha1_noanchor.so,chunkio_amd/lib/libchunkio_amd.so --rounds 5 --iters 10 > $OUT/ab_sha1_anchor.txt 2>&1 || { tail -20 $OUT/ab_sha1_anchor.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_sha1_anchor.txt | tail -8
timeout -k 10 200 python tools/sha1_clock.py $A/sha1_clock.so --copies 1,8 --iters 3 > $OUT/sha1_clock_anchor.txt 2>&1 || { tail -20 $OUT/sha1_clock_anchor.txt; exit 1; }
grep -v amdgpu.ids $OUT/sha1_clock_anchor.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_sha1.py > $OUT/pytest_sha1.txt 2>&1 || { tail -20 $OUT/pytest_sha1.txt; exit 1; }
tail -1 $OUT/pytest_sha1.txt
