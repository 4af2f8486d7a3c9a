#!/bin/bash
# Round-5 GPU session ac (and ag): the final-tree checks (GPU suite, smoke, sanitizers on
# the GPU route incl. the overlapped batched sync), a cfg2 rocprofv3 pair and the
# driver's default line.
set -u
O=gpurun_out/${1:-r05ac}
mkdir -p $O
export TMPDIR=/tmp
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1; step $? pytest
tail -1 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; step $? smoke
timeout -k 10 500 bash tools/asan_check.sh gpu > $O/asan_gpu.txt 2>&1; step $? asan-gpu
timeout -k 10 500 bash tools/asan_check.sh tsan-gpu > $O/tsan_gpu.txt 2>&1; step $? tsan-gpu
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg2 -o run --output-format csv -- \
    python3 bench.py --config cfg2 --steps 300 --warmup 200 --no-cpu --no-extra > $O/bench_prof_cfg2.json 2> $O/prof_cfg2.err
step $? prof_cfg2
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err; step $? default
echo all-done
