#!/bin/bash
# rocprofv3 kernel-trace summaries of the cfg4k (small-chunk kernel) and cfg5
# (SHA-1) bench legs.  Usage (GPU box, repo root): bash tools/prof_extra.sh TAG
set -u
TAG=${1:-extra}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg4k_$TAG -o run --output-format csv -- \
    python3 bench.py --config cfg4k --steps 300 --warmup 200 --no-cpu > gpurun_out/bench_prof_cfg4k_$TAG.json 2> gpurun_out/rocprof_cfg4k_$TAG.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sha1_$TAG -o run --output-format csv -- \
    python3 bench.py --config sha1 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_prof_sha1_$TAG.json 2> gpurun_out/rocprof_sha1_$TAG.err || exit $?
echo done
