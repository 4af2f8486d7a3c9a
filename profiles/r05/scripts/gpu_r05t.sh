#!/bin/bash
# Round-5 GPU session t: anti-camping grid (one workgroup fewer per 32 when
# every wave's range is a multiple of 16 steps up to 64) -- GPU suite, then
# interleaved A/B against CIO_GPU_ANTICAMP=0.
set -u
O=gpurun_out/${1:-r05t}
mkdir -p $O
export TMPDIR=/tmp
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1; step $? pytest
tail -2 $O/pytest_gpu.txt
timeout -k 10 700 python tools/ab_lib.py --libs chunkio_amd/lib/libchunkio_amd.so,chunkio_amd/lib/libchunkio_amd.so --env "CIO_GPU_ANTICAMP=0|" \
    --cfg k4x65536,k4x131072,k4x262144,k4x98304,cfg4k,cfg2,big --iters 30 --rounds 4 > $O/ab_anticamp.txt 2>&1; step $? ab
tail -1 $O/ab_anticamp.txt
echo all-done
