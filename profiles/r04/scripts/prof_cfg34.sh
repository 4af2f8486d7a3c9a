#!/bin/bash
# rocprofv3 kernel-trace summaries of the cfg3 and cfg4 (N = 1) bench legs,
# for tools/prof_pair.py.  Usage (GPU box, repo root): bash tools/prof_cfg34.sh TAG
set -u
TAG=${1:-c34}
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in cfg3 cfg4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${C}_$TAG -o run --output-format csv -- \
      python3 bench.py --config $C --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_prof_${C}_$TAG.json 2> gpurun_out/rocprof_${C}_$TAG.err || exit $?
done
echo done
