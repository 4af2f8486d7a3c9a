#!/bin/bash
# L64 layout everywhere: parity of every CRC GPU test in both layouts, then
# A/Bs: small kernel (cfg4k, 64K x 4 KiB), general stream kernel (cfg3), and
# the issue-ahead L64 stream kernel against the one-slot 4-sub-chain kernel.
set -u
OUT=gpurun_out/r03g; mkdir -p $OUT; export TMPDIR=/tmp
L=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_crc.py -v -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/pytest_l64.txt 2>&1 || { tail -30 $OUT/pytest_l64.txt; exit 1; }
tail -3 $OUT/pytest_l64.txt
timeout -k 10 300 python tools/ab_lib.py --libs $L,$L --env 'CIO_GPU_L64=0|CIO_GPU_L64=1' --cfg cfg4k,small,cfg3 --iters 100 --rounds 4 > $OUT/ab_l64_small_general.txt 2>&1 || exit $?
tail -1 $OUT/ab_l64_small_general.txt
timeout -k 10 400 python tools/ab_lib.py --libs $L,$L --env 'CIO_GPU_AHEAD=0,CIO_GPU_L64=0|CIO_GPU_L64=1' --cfg cfg2,mid,big --iters 200 --rounds 4 > $OUT/ab_l64_vs_oneslot.txt 2>&1 || exit $?
tail -1 $OUT/ab_l64_vs_oneslot.txt
