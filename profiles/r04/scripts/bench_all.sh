#!/bin/bash
# Every BASELINE config on one GPU (cfg2 default line, cfg3, cfg4 at N=1,
# SHA-1, end-to-end from host memory), one JSON line each.  Each GPU step has
# its own time limit; the script stops at the first fault/timeout.
# Usage (repo root, GPU box): bash tools/bench_all.sh [tag]
set -u
TAG=${1:-r01}
OUT=gpurun_out
mkdir -p $OUT
: > $OUT/bench_all_$TAG.jsonl
for cfg in cfg2 cfg4k cfg3 cfg4 sha1 e2e perf verify; do
  case $cfg in
    cfg3|cfg4) extra="--steps 100 --warmup 20 --no-cpu" ;;
    cfg4k) extra="--no-cpu" ;;
    sha1) extra="--steps 20 --warmup 3" ;;
    e2e) extra="--steps 10 --warmup 2" ;;
    perf) extra="--steps 3" ;;
    verify) extra="--steps 10 --warmup 2" ;;
    *) extra="--no-cpu" ;;
  esac
  timeout -k 10 600 python bench.py --config $cfg $extra >> $OUT/bench_all_$TAG.jsonl 2> $OUT/bench_all_${TAG}_$cfg.err
  rc=$?
  echo "[$cfg] rc=$rc"
  if [ $rc -ne 0 ]; then echo "stopping after $cfg"; exit $rc; fi
done
cat $OUT/bench_all_$TAG.jsonl
