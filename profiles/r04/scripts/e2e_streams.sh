#!/bin/bash
# Standalone e2e lines with k streams created before the pipeline's own
# (CIO_BENCH_PRE_STREAMS=k).  Usage: bash profiles/r04/scripts/e2e_streams.sh TAG k1 k2 ...
set -u
TAG=$1; shift; D=gpurun_out/$TAG; mkdir -p $D
for k in "$@"; do
  CIO_GPU_PIPE_TIMING=1 CIO_BENCH_PRE_STREAMS=$k timeout -k 10 150 python bench.py --config e2e --steps 30 --warmup 10 --no-cpu > $D/k$k.json 2> $D/k$k.err || exit $?
  python3 - "$D/k$k.json" "$k" <<'PY'
import json, sys
e = json.load(open(sys.argv[1]))
print(f"pre-streams {sys.argv[2]}: e2e staged {e['value']:7.2f} registered {e['registered_in_place']['value']:7.2f}")
PY
done
