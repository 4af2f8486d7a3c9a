#!/bin/bash
# A/B on the final stream kernel: per-step priority rotation on/off (CIO_GPU_PRIO).
set -u
OUT=gpurun_out/${1:-r03ze}; mkdir -p $OUT; export TMPDIR=/tmp
M=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 500 python tools/ab_lib.py --libs $M,$M,$M,$M --env 'CIO_GPU_PRIO=1|CIO_GPU_PRIO=0|CIO_GPU_PRIO=1|CIO_GPU_PRIO=0' --cfg cfg2,cfg4k,cfg3 --iters 100 --rounds 3 > $OUT/ab_prio_env.txt 2>&1 || { tail -20 $OUT/ab_prio_env.txt; exit 1; }
tail -1 $OUT/ab_prio_env.txt
