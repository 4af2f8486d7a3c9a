#!/bin/bash
# Copy/kernel timeline of the E2E leg (staged and registered host batches):
# rocprofv3 kernel + memory-copy trace, no counters.
set -u
OUT=gpurun_out/${1:-r03zg}; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/trace -o e2e -- \
  python bench.py --config e2e --steps 6 --warmup 2 --no-cpu > $OUT/bench_e2e.json 2> $OUT/bench_e2e.err || { tail -20 $OUT/bench_e2e.err; exit 1; }
find $OUT/trace -name "*.csv" | head -20
