#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel trace.  Each GPU step
# has its own time limit; the script stops at the first fault/timeout.
# Usage (from the repo root, on the GPU box): bash tools/gpu_check.sh [tag] [config] [notest]
set -u
TAG=${1:-r01}
CFG=${2:-cfg2}
NOTEST=${3:-}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
stop_if_fatal() {   # rc of a GPU step: 0 ok, 1 test failures (keep going), else stop
  local rc=$1 what=$2
  echo "[$what] rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal rc in $what, stopping"; exit "$rc"; fi
}
rocm-smi --showproductname > $OUT/gpu_info.txt 2>&1 || true
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.txt 2>&1
  stop_if_fatal $? pytest
  tail -5 $OUT/pytest_gpu_$TAG.txt
fi
timeout -k 10 400 python bench.py --config $CFG > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
stop_if_fatal $? bench
cat $OUT/bench_$TAG.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- \
    python3 bench.py --config $CFG --steps 300 --warmup 200 --no-cpu --no-extra > $OUT/bench_prof_$TAG.json 2> $OUT/rocprof_$TAG.err
stop_if_fatal $? rocprof
find $OUT/prof_$TAG -name "*stats*" | head
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmcf_$TAG -o run --output-format csv -- \
    python3 bench.py --config $CFG --steps 20 --warmup 20 --no-cpu --no-extra > /dev/null 2> $OUT/pmcf_$TAG.err
stop_if_fatal $? pmc_fetch
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcw_$TAG -o run --output-format csv -- \
    python3 bench.py --config $CFG --steps 20 --warmup 20 --no-cpu --no-extra > /dev/null 2> $OUT/pmcw_$TAG.err
stop_if_fatal $? pmc_write
python3 tools/pmc_traffic.py $OUT/pmcf_$TAG $OUT/pmcw_$TAG $CFG && cp profiles/pmc_$CFG.json $OUT/pmc_${CFG}_$TAG.json
