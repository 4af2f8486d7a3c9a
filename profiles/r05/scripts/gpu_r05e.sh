#!/bin/bash
# Round-5 GPU session e: the driver's default line on the final kernels,
# rocprofv3 kernel-trace pairs (cfg2 headline, cfg3), and an N = 4 rehearsal.
set -u
O=gpurun_out/r05e
mkdir -p $O
export TMPDIR=/tmp
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err; step $? default
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg2 -o run --output-format csv -- \
    python3 bench.py --config cfg2 --steps 300 --warmup 200 --no-cpu --no-extra > $O/bench_prof_cfg2.json 2> $O/prof_cfg2.err
step $? prof_cfg2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg3 -o run --output-format csv -- \
    python3 bench.py --config cfg3 --steps 10 --warmup 2 --no-cpu > $O/bench_prof_cfg3.json 2> $O/prof_cfg3.err
step $? prof_cfg3
CIO_BENCH_REHEARSE=1 timeout -k 10 900 python bench.py --gpus 4 > $O/bench_rehearse_n4.json 2> $O/bench_rehearse_n4.err
step $? n4
echo all-done
