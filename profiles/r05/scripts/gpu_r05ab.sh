#!/bin/bash
# Round-5 GPU session ab: async batched sync -- chunk-layer GPU tests, then the
# config-1 loop ceiling with the pipelined legs.
set -u
O=gpurun_out/${1:-r05ab}
mkdir -p $O
export TMPDIR=/tmp
step() { local rc=$1 what=$2; echo "[$what] rc=$rc"; if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_chunkfile.py tests/test_c_api.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest_chunk_gpu.txt 2>&1; step $? pytest_chunk
tail -1 $O/pytest_chunk_gpu.txt
timeout -k 10 500 python tools/perf_ceiling.py --rounds 6 > $O/perf_ceiling.txt 2>&1; step $? ceiling
tail -7 $O/perf_ceiling.txt
echo all-done
