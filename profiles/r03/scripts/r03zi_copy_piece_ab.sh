#!/bin/bash
# E2E staged host batches: fixed 1 MiB copy pieces (the old pool) against the
# adaptive piece size, interleaved, 4 passes; one process per run.
set -u
OUT=gpurun_out/${1:-r03zi}; mkdir -p $OUT; export TMPDIR=/tmp
: > $OUT/ab.txt
for pass in 1 2 3 4; do
for v in "old CIO_GPU_COPY_PIECE_KB=1024" "adaptive CIO_GPU_COPY_PIECE_KB=0" "adaptive_first8 CIO_GPU_STAGE_FIRST_MB=8"; do
  set -- $v
  env $2 timeout -k 10 120 python bench.py --config e2e --steps 30 --warmup 5 --no-cpu > $OUT/e2e_$1_$pass.json 2> $OUT/e2e_$1_$pass.err || { tail -5 $OUT/e2e_$1_$pass.err; exit 1; }
  python -c "
import json; l=json.loads(open('$OUT/e2e_$1_$pass.json').read().strip().splitlines()[-1])
r=l['registered_in_place']; p=l['pipe_legs_last_call']['staged']
print('pass $pass %-16s staged %.2f GB/s (%.3f ms), registered %.2f, h2d %.1f, legs total %.2f copy %.2f wait %.2f' % ('$1', l['value'], l['ms_per_step'], r['value'], l['breakdown']['pinned_h2d_GBps'], p['total_ms'], p['copy_ms'], p['slot_wait_ms']))
" | tee -a $OUT/ab.txt
done
done
