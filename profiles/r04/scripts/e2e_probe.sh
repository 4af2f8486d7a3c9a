#!/bin/bash
# E2E host-pipeline probe: the driver's default line and a standalone e2e
# line, each with per-call pipeline legs on stderr (CIO_GPU_PIPE_TIMING=1).
# Usage: bash profiles/r04/scripts/e2e_probe.sh TAG
set -u
TAG=$1; D=gpurun_out/$TAG; mkdir -p $D
CIO_GPU_PIPE_TIMING=1 timeout -k 10 400 python bench.py > $D/default.json 2> $D/default.err || exit $?
CIO_GPU_PIPE_TIMING=1 timeout -k 10 150 python bench.py --config e2e --steps 30 --warmup 10 --no-cpu > $D/e2e.json 2> $D/e2e.err || exit $?
python3 - "$D" <<'PY'
import json, sys
d = sys.argv[1]
a = json.load(open(f"{d}/default.json"))
e = a["other_configs"]["e2e"]
print("default line: cfg2 frac", a["roofline"]["frac"], "e2e staged", e["value"], "registered", e["registered_in_place"]["value"])
b = json.load(open(f"{d}/e2e.json"))
print("standalone : e2e staged", b["value"], "registered", b["registered_in_place"]["value"])
PY
