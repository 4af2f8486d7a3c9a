#!/bin/bash
# Host pipeline: one copy stream for every data DMA (new) against DMAs on the slot streams (pipe_old.so).
set -u
OUT=gpurun_out/r03l; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
for r in 1 2 3; do
  for tag in old new; do
    if [ $tag = old ]; then export CIO_AMD_LIB=chunkio_amd/lib/ab/pipe_old.so; else unset CIO_AMD_LIB; fi
    timeout -k 10 120 python bench.py --config e2e --steps 30 --warmup 10 --no-cpu > $OUT/e2e_${tag}_$r.json 2>/dev/null || exit $?
    timeout -k 10 200 python bench.py --config verify --steps 3 --warmup 1 --no-cpu > $OUT/verify_${tag}_$r.json 2>/dev/null || exit $?
  done
done
unset CIO_AMD_LIB
python3 - <<'PY'
import json
for tag in ("old", "new"):
    for r in (1, 2, 3):
        d = json.loads(open(f"gpurun_out/r03l/e2e_{tag}_{r}.json").read().strip().splitlines()[-1])
        v = json.loads(open(f"gpurun_out/r03l/verify_{tag}_{r}.json").read().strip().splitlines()[-1])
        pl = d.get("pipe_legs_last_call", {})
        print(tag, r, "staged", d["value"], "registered", d["registered_in_place"]["value"],
              "h2d", d["breakdown"]["pinned_h2d_GBps"], "verify", v["value"], d["check"])
PY
