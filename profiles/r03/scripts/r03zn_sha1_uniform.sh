#!/bin/bash
# SHA-1: wave-uniform block counts (scalar group loops) on top of the round-order
# anchor, against the anchor alone (-DCIO_SHA1_NO_UNIFORM), interleaved; SHA-1 GPU tests.
set -u
OUT=gpurun_out/${1:-r03zn}; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
timeout -k 10 300 python tools/sha1_ab.py --libs $A/sha1_anchor_only.so,chunkio_amd/lib/libchunkio_amd.so --rounds 5 --iters 10 > $OUT/ab_sha1_uniform.txt 2>&1 || { tail -20 $OUT/ab_sha1_uniform.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_sha1_uniform.txt | tail -4
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_sha1.py > $OUT/pytest_sha1.txt 2>&1 || { tail -20 $OUT/pytest_sha1.txt; exit 1; }
tail -1 $OUT/pytest_sha1.txt
