#!/bin/bash
# The CRC GPU tests under the library's other kernel selections: issue-ahead
# off (one-slot stream kernel everywhere) and the small-chunk kernel off (every
# batch on the stream kernel); the chunk-layer tests with every CRC on the GPU.
set -u
OUT=gpurun_out/${1:-r03zf}; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift; env "$@" timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu -p no:cacheprovider $T > $OUT/pytest_$name.txt 2>&1; local rc=$?; echo "[$name] rc=$rc $(tail -1 $OUT/pytest_$name.txt)"; return $rc; }
T=tests/test_gpu_crc.py
run ahead0 CIO_GPU_AHEAD=0 && run small0 CIO_GPU_SMALL=0 && T="tests/test_chunkfile.py tests/test_c_api.py" && run cpumax0 CIOA_CPU_CRC_MAX=0
