#!/bin/bash
# Round-5 GPU session c: counter list, sanitizers on the GPU route (narrowed
# TSan suppressions), cfg3 traffic attribution (raw vs 4 KiB-rounded geometry).
set -u
O=gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
(cd /tmp && timeout -s KILL 100 rocprofv3 -L > $R/$O/counters.txt 2>&1); step $? list
timeout -k 10 400 bash tools/asan_check.sh gpu > $O/asan_gpu.txt 2>&1; step $? asan-gpu
timeout -k 10 400 bash tools/asan_check.sh tsan-gpu > $O/tsan_gpu.txt 2>&1; step $? tsan-gpu
for G in raw r4096; do
  if [ $G = r4096 ]; then export CIO_BENCH_CFG3_ROUND=4096; else unset CIO_BENCH_CFG3_ROUND; fi
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf_cfg3_$G -o run --output-format csv -- \
      python3 bench.py --config cfg3 --steps 4 --warmup 1 --no-cpu --no-extra > $O/bench_cfg3_$G.json 2> $O/pmcf_cfg3_$G.err
  step $? fetch_$G
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw_cfg3_$G -o run --output-format csv -- \
      python3 bench.py --config cfg3 --steps 4 --warmup 1 --no-cpu --no-extra > /dev/null 2> $O/pmcw_cfg3_$G.err
  step $? write_$G
done
# the same raw cfg3 geometry on the 128-byte-head build (CIO_HEAD_ALIGN=128)
unset CIO_BENCH_CFG3_ROUND
CIO_AMD_LIB=chunkio_amd/lib/ab/al128.so timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf_cfg3_al128 -o run --output-format csv -- \
    python3 bench.py --config cfg3 --steps 4 --warmup 1 --no-cpu --no-extra > $O/bench_cfg3_al128.json 2> $O/pmcf_cfg3_al128.err
step $? fetch_al128
echo all-done
