#!/bin/bash
# Round-5 GPU session m: rocprofv3 pairs for cfg4k, cfg4 and SHA-1 on the final
# kernels, a request-size PMC pass for cfg4, and the default line.
set -u
O=gpurun_out/${1:-r05m}
mkdir -p $O
export TMPDIR=/tmp
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg4k -o run --output-format csv -- \
    python3 bench.py --config cfg4k --steps 300 --warmup 200 --no-cpu > $O/bench_prof_cfg4k.json 2> $O/prof_cfg4k.err
step $? prof_cfg4k
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg4 -o run --output-format csv -- \
    python3 bench.py --config cfg4 --steps 20 --warmup 5 --no-cpu > $O/bench_prof_cfg4.json 2> $O/prof_cfg4.err
step $? prof_cfg4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_sha1 -o run --output-format csv -- \
    python3 bench.py --config sha1 --steps 20 --warmup 3 --no-cpu > $O/bench_prof_sha1.json 2> $O/prof_sha1.err
step $? prof_sha1
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
timeout -s KILL 120 rocprofv3 --pmc $C -d $O/pmcq_cfg4 -o run --output-format csv -- \
    python3 bench.py --config cfg4 --steps 4 --warmup 1 --no-cpu --no-extra > /dev/null 2> $O/pmcq_cfg4.err
step $? reqsize_cfg4
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err; step $? default
echo all-done
