#!/bin/bash
# Round-5 GPU session d: the GPU suite against the 128-byte-head build, and
# in-process A/Bs: head alignment (cfg3, mixed, 4 MiB) and the small kernel's
# fold.
set -u
O=gpurun_out/r05d
mkdir -p $O
export TMPDIR=/tmp
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
L=chunkio_amd/lib/libchunkio_amd.so
CIO_AMD_LIB=chunkio_amd/lib/ab/al128.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest_gpu_al128.txt 2>&1; step $? pytest_al128
tail -2 $O/pytest_gpu_al128.txt
timeout -k 10 500 python tools/ab_lib.py --libs $L,chunkio_amd/lib/ab/al128.so \
    --cfg cfg3,mid,big --iters 20 --rounds 4 > $O/ab_head_align.txt 2>&1; step $? ab_align
# small-kernel fold A/B: shipped 4-sub-chain layout,
# L64 layout, L64 + nibble-table fold; then the fold priced (wrong CRCs)
L=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 400 python tools/ab_lib.py --libs $L,$L,chunkio_amd/lib/ab/nibfold.so --env "|CIO_GPU_L64=1|CIO_GPU_L64=1" \
    --cfg cfg4k,small --iters 40 --rounds 5 > $O/ab_small_nibfold.txt 2>&1; step $? ab_nibfold
timeout -k 10 400 python tools/ab_lib.py --libs $L,chunkio_amd/lib/ab/nofold.so --no-check \
    --cfg cfg4k --iters 40 --rounds 4 > $O/ab_small_nofold.txt 2>&1; step $? ab_nofold
echo all-done
