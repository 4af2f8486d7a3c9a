#!/bin/bash
# Default line reduced to its cfg2 leg + the e2e leg, with parts of the cfg2
# leg switched off.  Each argument: "NAME|ENV=..,ENV=..|bench flags".
# Usage: bash profiles/r04/scripts/e2e_bisect.sh TAG "full||" "nocpu||--no-cpu" ...
set -u
TAG=$1; shift; D=gpurun_out/$TAG; mkdir -p $D
for spec in "$@"; do
  IFS='|' read -r name envs flags <<< "$spec"
  ( export CIO_BENCH_LEGS=e2e; for kv in ${envs//,/ }; do export "$kv"; done
    timeout -k 10 300 python bench.py $flags > $D/$name.json 2> $D/$name.err ) || exit $?
  python3 - "$D/$name.json" "$name" <<'PY'
import json, sys
a = json.load(open(sys.argv[1]))
e = a["other_configs"]["e2e"]
print(f"{sys.argv[2]:>12}: e2e staged {e['value']:7.2f} registered {e['registered_in_place']['value']:7.2f}")
PY
done
