#!/bin/bash
# Round-5 GPU session n: the small-chunk kernel (cfg4k) priced by ablation:
# shipped, no lane fold (EXP=1), no LDS CRC (EXP=2), neither (EXP=3); wrong
# CRCs in the ablations, timing only.  Each through bench.py --config cfg4k
# (kernel event time and the same-grid read-only stream), interleaved twice.
set -u
O=gpurun_out/${1:-r05n}
mkdir -p $O
export TMPDIR=/tmp
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
for r in 1 2; do
  for v in product nofold exp2 exp3; do
    if [ $v = product ]; then L=chunkio_amd/lib/libchunkio_amd.so; else L=chunkio_amd/lib/ab/$v.so; fi
    CIO_AMD_LIB=$L timeout -k 10 120 python bench.py --config cfg4k --steps 300 --warmup 100 --no-cpu \
        > $O/cfg4k_${v}_$r.json 2> $O/cfg4k_${v}_$r.err; step $? ${v}_$r
  done
done
echo all-done
