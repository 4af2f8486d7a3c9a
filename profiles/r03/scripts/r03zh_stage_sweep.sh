#!/bin/bash
# E2E staged/registered host batches against the staging schedule knobs
# (CIO_GPU_STAGE_MB = slot size, CIO_GPU_STAGE_FIRST_MB = first group), two passes
# interleaved; one process per setting (the knobs are read once per process).
set -u
OUT=gpurun_out/${1:-r03zh}; mkdir -p $OUT; export TMPDIR=/tmp
: > $OUT/sweep.txt
for pass in 1 2; do
for cfg in "64 4" "16 16" "8 8" "16 4" "32 32" "4 4"; do
  set -- $cfg
  CIO_GPU_STAGE_MB=$1 CIO_GPU_STAGE_FIRST_MB=$2 timeout -k 10 120 python bench.py --config e2e --steps 20 --warmup 5 --no-cpu > $OUT/e2e_$1_$2_$pass.json 2> $OUT/e2e_$1_$2_$pass.err || { tail -5 $OUT/e2e_$1_$2_$pass.err; exit 1; }
  python -c "
import json,sys; l=json.loads(open('$OUT/e2e_$1_$2_$pass.json').read().strip().splitlines()[-1])
r=l['registered_in_place']; p=l.get('pipe_legs_last_call',{})
print('pass $pass stage $1 first $2: staged %.1f GB/s (%.2f ms), registered %.1f GB/s, h2d %.1f | staged legs %s' % (l['value'], l['ms_per_step'], r['value'], l['breakdown']['pinned_h2d_GBps'], {k: round(v,2) for k,v in p.get('staged',{}).items()}))
" | tee -a $OUT/sweep.txt
done
done
