#!/bin/bash
# Which earlier leg of the default line slows its e2e leg: the default line
# with only some legs, in a given order (CIO_BENCH_LEGS), e2e values printed.
# Usage: bash profiles/r04/scripts/e2e_order.sh TAG "e2e" "cfg3,e2e" ...
set -u
TAG=$1; shift; D=gpurun_out/$TAG; mkdir -p $D
i=0
for legs in "$@"; do
  i=$((i+1))
  CIO_BENCH_LEGS=$legs timeout -k 10 300 python bench.py > $D/run$i.json 2> $D/run$i.err || exit $?
  python3 - "$D/run$i.json" "$legs" <<'PY'
import json, sys
a = json.load(open(sys.argv[1]))
e = a["other_configs"]["e2e"]
print(f"{sys.argv[2]:>24}: e2e staged {e['value']:7.2f} registered {e['registered_in_place']['value']:7.2f} "
      f"h2d_reg {e['registered_in_place']['h2d_from_registered_pages_GBps']} pinned {e['breakdown']['pinned_h2d_GBps']}")
PY
done
