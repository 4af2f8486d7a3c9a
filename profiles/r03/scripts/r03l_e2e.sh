#!/bin/bash
# E2E host pipeline timeline: kernel + memory-copy trace of the e2e bench config.
set -u
OUT=gpurun_out/r03l; mkdir -p $OUT; export TMPDIR=/tmp
CIO_GPU_PIPE_TIMING=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/e2e -o run --output-format csv -- \
    python3 bench.py --config e2e --steps 5 --warmup 2 --no-cpu --no-extra > $OUT/e2e.json 2> $OUT/e2e.err || exit $?
grep batch_host $OUT/e2e.err | tail -4
find $OUT/e2e -name "*.csv" | head
