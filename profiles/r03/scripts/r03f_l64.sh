#!/bin/bash
# L64 layout: parity first, then the interleaved A/B against the 4-sub-chain
# issue-ahead kernel (both forced on with CIO_GPU_AHEAD=1).
set -u
OUT=gpurun_out/r03f; mkdir -p $OUT; export TMPDIR=/tmp
L=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_crc.py -k "issue_ahead or cfg2_full or cfg4" -v -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/pytest_l64.txt 2>&1 || { tail -30 $OUT/pytest_l64.txt; exit 1; }
tail -3 $OUT/pytest_l64.txt
timeout -k 10 400 python tools/ab_lib.py --libs $L,$L --env 'CIO_GPU_AHEAD=1,CIO_GPU_L64=0|CIO_GPU_AHEAD=1,CIO_GPU_L64=1' --cfg ${CFGS:-cfg2,mid,big} --iters 200 --rounds 4 > $OUT/ab_l64.txt 2>&1 || exit $?
tail -1 $OUT/ab_l64.txt
