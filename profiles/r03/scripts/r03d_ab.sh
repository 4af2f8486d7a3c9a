set -u
OUT=gpurun_out/r03d; mkdir -p $OUT; export TMPDIR=/tmp
L=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 300 python tools/ab_lib.py --libs $L,chunkio_amd/lib/ab/halfrep.so --cfg cfg2,big,cfg4k --iters 200 --rounds 3 > $OUT/ab_halfrep.txt 2>&1 || exit $?
timeout -k 10 400 python tools/ab_lib.py --libs $L,$L --env 'CIO_GPU_AHEAD=0|CIO_GPU_AHEAD=1' --cfg cfg2,mid,big --iters 200 --rounds 4 > $OUT/ab_ahead2.txt 2>&1 || exit $?
echo done
