#!/bin/bash
# Round-5 GPU session d: the GPU suite on the product (128-byte heads), the
# head-alignment A/B against the round-4 16-byte heads, the small kernel's fold
# A/B, and request-size PMC passes (no x2 calibration).
set -u
O=gpurun_out/r05d
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
L=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1; step $? pytest
tail -2 $O/pytest_gpu.txt
timeout -k 10 500 python tools/ab_lib.py --libs $L,chunkio_amd/lib/ab/al16.so \
    --cfg cfg3,mid,big --iters 20 --rounds 4 > $O/ab_head_align.txt 2>&1; step $? ab_align
tail -1 $O/ab_head_align.txt
timeout -k 10 400 python tools/ab_lib.py --libs $L,$L,chunkio_amd/lib/ab/nibfold.so --env "|CIO_GPU_L64=1|CIO_GPU_L64=1" \
    --cfg cfg4k,small --iters 40 --rounds 5 > $O/ab_small_nibfold.txt 2>&1; step $? ab_nibfold
tail -1 $O/ab_small_nibfold.txt
timeout -k 10 400 python tools/ab_lib.py --libs $L,chunkio_amd/lib/ab/nofold.so --no-check \
    --cfg cfg4k --iters 40 --rounds 4 > $O/ab_small_nofold.txt 2>&1; step $? ab_nofold
tail -1 $O/ab_small_nofold.txt
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
for CFG in cfg2 cfg3 cfg4k; do
  (cd $R && timeout -s KILL 120 rocprofv3 --pmc $C -d $O/pmcq_$CFG -o run --output-format csv -- \
      python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu --no-extra > /dev/null 2> $O/pmcq_$CFG.err)
  step $? reqsize_$CFG
done
CIO_AMD_LIB=chunkio_amd/lib/ab/al16.so timeout -s KILL 120 rocprofv3 --pmc $C -d $O/pmcq_cfg3_al16 -o run \
    --output-format csv -- python3 bench.py --config cfg3 --steps 10 --warmup 2 --no-cpu --no-extra > /dev/null 2> $O/pmcq_cfg3_al16.err
step $? reqsize_cfg3_al16
echo all-done
