#!/bin/bash
# Round-5 GPU session ae: GPU suite + smoke on the final library, and the N = 2
# rehearsal (two ranks on the one GPU) of the driver's command with the final
# bench.py (perf leg with pipelined_sync).
set -u
O=gpurun_out/${1:-r05ae}
mkdir -p $O
export TMPDIR=/tmp
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1; step $? pytest
tail -1 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; step $? smoke
CIO_BENCH_REHEARSE=1 timeout -k 10 700 python bench.py --gpus 2 > $O/bench_rehearse_n2.json 2> $O/bench_rehearse_n2.err; step $? rehearse_n2
echo all-done
