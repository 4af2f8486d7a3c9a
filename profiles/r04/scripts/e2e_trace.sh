#!/bin/bash
# Copy/kernel timelines of the standalone e2e line with and without a prior
# 34.4 GB device allocation (CIO_BENCH_PRE_ALLOC_GB): rocprofv3 kernel +
# memory-copy trace, no counters.  Usage: bash profiles/r04/scripts/e2e_trace.sh TAG
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
export TMPDIR=/tmp
for v in base alloc34 alloc34after; do
  if [ $v = alloc34 ]; then export CIO_BENCH_PRE_ALLOC_GB=34.4; fi
  if [ $v = alloc34after ]; then export CIO_BENCH_ALLOC_AFTER_WARM=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace_$v -o e2e -- \
    python bench.py --config e2e --steps 6 --warmup 2 --no-cpu > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { tail -20 $OUT/bench_$v.err; exit 1; }
done
find $OUT -name "*.csv"
