#!/bin/bash
# Final-tree GPU check: smoke, GPU tests, default bench line (wall time
# recorded), a 2-rank rehearsal of the N>1 path on one GPU, rocprofv3 kernel
# trace of the cfg2 line.  Each step has its own time limit; stops at the
# first failure.  Usage: bash tools/final_check.sh TAG [notest]
set -u
TAG=${1:-final}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${2:-}" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 || exit $?
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.txt 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_$TAG.txt; [ $rc -ne 0 ] && exit $rc
fi
t0=$(date +%s.%N)
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
t1=$(date +%s.%N)
python3 -c "print('default bench wall seconds: %.1f' % ($t1 - $t0))" | tee gpurun_out/bench_wall_$TAG.txt
CIO_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 200 --warmup 50 > gpurun_out/bench_rehearse_n2_$TAG.json 2> gpurun_out/bench_rehearse_n2_$TAG.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --config cfg2 --steps 300 --warmup 200 --no-cpu --no-extra > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/rocprof_$TAG.err || exit $?
echo done
