#!/bin/bash
# A/B: the CRC kernels' data loads with the default cache policy instead of nt.
set -u
OUT=gpurun_out/${1:-r03z2}; mkdir -p $OUT; export TMPDIR=/tmp
A=chunkio_amd/lib/ab
timeout -k 10 500 python tools/ab_lib.py --libs $A/crc_base.so,$A/crc_ld_plain.so,$A/crc_base.so,$A/crc_ld_plain.so --cfg cfg2,cfg4k,big --iters 200 --rounds 3 > $OUT/ab_ld_policy.txt 2>&1 || { tail -20 $OUT/ab_ld_policy.txt; exit 1; }
tail -2 $OUT/ab_ld_policy.txt
