#!/bin/bash
# Round-3 GPU session: smoke, GPU tests, the driver's default bench line, the
# driver's N-GPU command form rehearsed on one GPU (spawn path, no launcher
# env), the one-chunk latency crossover, and a rocprofv3 kernel trace of every
# bench line's kernel paired with that run's own line.  Each GPU step has its
# own time limit; the script stops at the first failure.
# Usage (GPU box, repo root): bash tools/r03_check.sh TAG [PHASES]
#   PHASES: comma list of test,ab,bench,spawn,cross,rsdyn,prof,pmc,pmc4k (default: test,ab,bench,spawn,cross,prof)
#   env PROF_CFGS=cfg2,sha1 limits the prof phase; PMC_CFGS the pmc phase
set -u
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {   # step NAME TIMEOUT CMD... : run, stop the script on any failure
  local name=$1 t=$2; shift 2
  local t0=$(date +%s.%N)
  timeout -k 10 $t "$@"
  local rc=$?
  echo "[$name] rc=$rc $(python3 -c "print('%.1f s' % ($(date +%s.%N) - $t0))")" | tee -a $OUT/steps.txt
  # pytest rc 1 = some tests failed (the GPU is fine): keep going; anything else stops
  if [ $rc -ne 0 ] && ! { [ "$name" = pytest ] && [ $rc -eq 1 ]; }; then exit $rc; fi
  return 0
}
PH=",${2:-test,ab,bench,spawn,cross,prof},"
has() { [[ "$PH" == *",$1,"* ]]; }
python3 -c "import sys; sys.path.insert(0, '.'); import bench; print('visible_gpus', bench.visible_gpus())" > $OUT/visible.txt 2>&1
python3 -c "import torch; print('torch device_count', torch.cuda.device_count())" >> $OUT/visible.txt 2>&1
if has test; then
  step smoke 300 bash -c "python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.txt 2>&1"
  step pytest 900 bash -c "python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1"
  tail -3 $OUT/pytest_gpu.txt
fi
has ab && step ab_ahead 400 bash -c "python tools/ab_lib.py --libs chunkio_amd/lib/libchunkio_amd.so,chunkio_amd/lib/libchunkio_amd.so --env 'CIO_GPU_AHEAD=0|CIO_GPU_AHEAD=1' --cfg cfg2,big --iters 200 --rounds 4 > $OUT/ab_ahead.txt 2>&1"
has bench && step bench_default 400 bash -c "python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err"
has spawn && step spawn_n2 400 bash -c "CIO_BENCH_REHEARSE=1 python bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/bench_spawn_n2.json 2> $OUT/bench_spawn_n2.err"
has spawn && step spawn_n4 500 bash -c "CIO_BENCH_REHEARSE=1 python bench.py --gpus 4 --steps 20 --warmup 5 > $OUT/bench_spawn_n4.json 2> $OUT/bench_spawn_n4.err"
has cross && step crossover 300 python tools/crossover.py $OUT/crossover.txt
has rsdyn && step rs_dyn 300 bash -c "python tools/rs_dyn_probe.py 4 '${RSDYN:-static;100,4,64;150,4,64;200,4,64;150,2,64;150,8,64;150,4,256;300,4,64}' > $OUT/rs_dyn_probe.txt 2>&1"
has pmc4k && step pmc_cfg4k 300 bash tools/pmc_configs.sh cfg4k
if has prof; then
  # rocprofv3 kernel traces, each of one bench line (the default line's legs, same K/W)
  for spec in "cfg2 20 5 crc32_stream_kernel 20" "cfg2 300 200 crc32_stream_kernel 100" \
              "cfg4k 200 50 crc32_small_kernel 100" "cfg4 20 5 crc32_stream_kernel 20" \
              "cfg3 5 2 crc32_stream_kernel 5" "sha1 10 2 sha1_kernel 0"; do
    set -- $spec
    cfg=$1; k=$2; w=$3; kern=$4; iso=$5
    [[ ",${PROF_CFGS:-$cfg}," == *",$cfg,"* ]] || continue
    d=$OUT/prof_${cfg}_k$k
    step prof_${cfg}_k$k 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
        python3 bench.py --config $cfg --steps $k --warmup $w --no-cpu --no-extra > $d.json 2> $d.err
    python3 tools/prof_pair.py $d.json $(find $d -name "run_kernel_trace.csv" | head -1) $kern $iso > $d.pair.json
  done
fi
if has pmc; then
  # HBM traffic of the final kernels (separate FETCH / WRITE passes)
  step pmc 600 bash tools/pmc_configs.sh ${PMC_CFGS:-cfg2 cfg3 cfg4 cfg4k}
fi
echo done
