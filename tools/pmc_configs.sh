#!/bin/bash
# PMC HBM traffic (FETCH_SIZE and WRITE_SIZE, separate passes) of the CRC
# kernel for the given bench configs -> profiles/pmc_<cfg>.json (read by
# bench.py for roofline.traffic).  Run on the GPU box from the repo root:
#   bash tools/pmc_configs.sh cfg3 cfg4
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for CFG in "$@"; do
  case $CFG in
    cfg3) ALGO=39748485057; STEPS=4; WARM=1 ;;
    cfg4) ALGO=34359738368; STEPS=4; WARM=1 ;;
    cfg4k) ALGO=419430400; STEPS=20; WARM=20 ;;
    sha1) ALGO=419430400; STEPS=5; WARM=1 ;;
    *) ALGO=419430400; STEPS=20; WARM=20 ;;
  esac
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmcf_$CFG -o run --output-format csv -- \
      python3 bench.py --config $CFG --steps $STEPS --warmup $WARM --no-cpu --no-extra > /dev/null 2> $OUT/pmcf_$CFG.err
  rc=$?; echo "[$CFG fetch] rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmcw_$CFG -o run --output-format csv -- \
      python3 bench.py --config $CFG --steps $STEPS --warmup $WARM --no-cpu --no-extra > /dev/null 2> $OUT/pmcw_$CFG.err
  rc=$?; echo "[$CFG write] rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 tools/pmc_traffic.py $OUT/pmcf_$CFG $OUT/pmcw_$CFG $CFG --algo $ALGO && cp profiles/pmc_$CFG.json $OUT/pmc_$CFG.json || exit 1
done
