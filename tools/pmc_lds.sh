#!/bin/bash
# LDS / VALU activity of the cfg2 kernel (one rocprofv3 --pmc pass of SQ
# counters, no tracing).  Usage (GPU box, repo root): bash tools/pmc_lds.sh TAG
set -u
TAG=${1:-lds}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD \
    -d gpurun_out/pmc_lds_$TAG -o run --output-format csv -- \
    python3 bench.py --config cfg2 --steps 20 --warmup 20 --no-cpu --no-extra > /dev/null 2> gpurun_out/pmc_lds_$TAG.err
rc=$?; echo "rc=$rc"; exit $rc
