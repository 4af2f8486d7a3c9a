#!/bin/bash
# One GPU session on the box, as a list of steps run in order; the session
# stops at the first step that fails, times out or faults (no retries).
#
# usage (repo root, on the GPU box):
#   bash tools/gpu_session.sh TAG STEP [STEP ...]
# steps:
#   tests[:PYTEST_ARGS]     pytest -m gpu (PYTEST_ARGS: extra args, '+' for spaces,
#                           e.g. tests:tests/test_gpu_sha1.py or tests:-k+sha1)
#   smoke                   __graft_entry__.smoke()
#   bench[:ARGS]            python bench.py ARGS ('+' for spaces) -> bench_<n>.json
#   prof:CFG:STEPS:WARMUP[:ARGS]
#                           rocprofv3 --kernel-trace --stats of bench.py --config CFG
#   pmc:CFG:COUNTERS        one rocprofv3 --pmc pass (COUNTERS comma-separated)
#   traffic:CFG             FETCH_SIZE and WRITE_SIZE passes + tools/pmc_traffic.py
#   py:SCRIPT[:ARGS]        python SCRIPT ARGS (a probe or measurement tool)
# Output goes to gpurun_out/TAG/.  Every step has its own time limit.
set -u
TAG=${1:?tag}
shift
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
n=0
stop_if_failed() {
  local rc=$1 what=$2
  echo "[$what] rc=$rc"
  if [ "$rc" -ne 0 ]; then echo "stop after $what"; exit "$rc"; fi
}
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  rest=""
  [ "$kind" != "$step" ] && rest=${step#*:}
  case $kind in
    tests)
      args=${rest//+/ }
      timeout -k 10 900 python -u -m pytest ${args:-tests} -m gpu -x -v -p no:cacheprovider \
          --timeout 120 --timeout-method thread > "$O/pytest_$n.txt" 2>&1
      rc=$?; tail -3 "$O/pytest_$n.txt"; stop_if_failed $rc "tests $args" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$n.txt" 2>&1
      rc=$?; tail -3 "$O/smoke_$n.txt"; stop_if_failed $rc smoke ;;
    bench)
      args=${rest//+/ }
      timeout -k 10 600 python bench.py $args > "$O/bench_$n.json" 2> "$O/bench_$n.err"
      rc=$?; cat "$O/bench_$n.json"; stop_if_failed $rc "bench $args" ;;
    prof)
      IFS=: read -r cfg steps warm args <<< "$rest"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof_${cfg}_$n" -o run --output-format csv -- \
          python3 bench.py --config "$cfg" --steps "${steps:-300}" --warmup "${warm:-200}" --no-cpu --no-extra ${args//+/ } \
          > "$O/bench_prof_${cfg}_$n.json" 2> "$O/prof_${cfg}_$n.err"
      stop_if_failed $? "prof $cfg" ;;
    pmc)
      IFS=: read -r cfg counters <<< "$rest"
      timeout -s KILL 120 rocprofv3 --pmc ${counters//,/ } -d "$O/pmc_${cfg}_$n" -o run --output-format csv -- \
          python3 bench.py --config "$cfg" --steps 4 --warmup 1 --no-cpu --no-extra > /dev/null 2> "$O/pmc_${cfg}_$n.err"
      stop_if_failed $? "pmc $cfg" ;;
    traffic)
      cfg=$rest
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/pmcf_$cfg" -o run --output-format csv -- \
          python3 bench.py --config "$cfg" --steps 20 --warmup 20 --no-cpu --no-extra > /dev/null 2> "$O/pmcf_$cfg.err"
      stop_if_failed $? "pmc FETCH_SIZE $cfg"
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/pmcw_$cfg" -o run --output-format csv -- \
          python3 bench.py --config "$cfg" --steps 20 --warmup 20 --no-cpu --no-extra > /dev/null 2> "$O/pmcw_$cfg.err"
      stop_if_failed $? "pmc WRITE_SIZE $cfg"
      python3 tools/pmc_traffic.py "$O/pmcf_$cfg" "$O/pmcw_$cfg" "$cfg" && cp "profiles/pmc_$cfg.json" "$O/" ;;
    py)
      IFS=: read -r script args <<< "$rest"
      timeout -k 10 600 python -u "$script" ${args//+/ } > "$O/py_$n.txt" 2>&1
      rc=$?; tail -5 "$O/py_$n.txt"; stop_if_failed $rc "py $script" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo all-done
