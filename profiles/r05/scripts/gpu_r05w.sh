#!/bin/bash
# Round-5 GPU session w: isolate the ab_lib cfg2 timing failure seen after
# c64kx32768 (session v).
set -u
O=gpurun_out/${1:-r05w}
mkdir -p $O
export TMPDIR=/tmp
L=chunkio_amd/lib/libchunkio_amd.so
timeout -k 10 200 python tools/ab_lib.py --libs $L --cfg cfg2 --iters 40 --rounds 2 --warm-s 0.5 > $O/a_cfg2.txt 2>&1; echo "a rc=$?"
tail -1 $O/a_cfg2.txt | cut -c1-300
timeout -k 10 200 python tools/ab_lib.py --libs $L --cfg cfg4k,cfg2 --iters 40 --rounds 2 --warm-s 0.5 > $O/b_cfg4k_cfg2.txt 2>&1; echo "b rc=$?"
tail -1 $O/b_cfg4k_cfg2.txt | cut -c1-300
timeout -k 10 200 python tools/ab_lib.py --libs $L --cfg cfg2 --iters 40 --rounds 2 --warm-s 0 > $O/c_cfg2_nowarm.txt 2>&1; echo "c rc=$?"
tail -1 $O/c_cfg2_nowarm.txt | cut -c1-300
echo all-done
