#!/bin/bash
# GPU A/B session: GPU parity tests on the in-tree library, then an in-process
# A/B of candidate libraries.  Usage: bash tools/gpu_ab.sh TAG LIBS ENVS CFGS
set -u
TAG=$1; LIBS=$2; ENVS=$3; CFGS=${4:-cfg2,big,cfg3,small}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python tools/ab_lib.py --libs $LIBS --env "$ENVS" --cfg $CFGS --iters 40 --rounds 4 > gpurun_out/ab_$TAG.txt 2>&1
rc=$?; echo "ab rc=$rc"; tail -1 gpurun_out/ab_$TAG.txt; exit $rc
