#!/bin/bash
# Round-5 GPU session v: anti-camping A/B with warm clocks and ABBA order
# (lib1 and lib2 are the same default plan where the range cap does not
# differ: an A/A check of the method).
set -u
O=gpurun_out/${1:-r05v}
mkdir -p $O
export TMPDIR=/tmp
L=chunkio_amd/lib/libchunkio_amd.so
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
timeout -k 10 700 python tools/ab_lib.py --libs $L,$L,$L --env "CIO_GPU_ANTICAMP=0||CIO_GPU_ANTICAMP_MAX=1023" \
    --cfg k4x65536,k4x131072,k4x262144,c64kx4096,c64kx8192,c64kx16384,k4x524288,c64kx32768,cfg2,cfg4k,cfg3,big \
    --iters 40 --rounds 6 --warm-s 1.5 > $O/ab_anticamp_abba.txt 2>&1; step $? ab
tail -1 $O/ab_anticamp_abba.txt
echo all-done
