#!/bin/bash
# Host pipeline: staging slots 2 / 3 (default) / 4 / 6, runs alternated.
set -u
OUT=gpurun_out/r03l; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2 3; do
  for tag in s2 s3 s4 s6; do
    if [ $tag = s3 ]; then unset CIO_AMD_LIB; else export CIO_AMD_LIB=chunkio_amd/lib/ab/pipe_$tag.so; fi
    timeout -k 10 120 python bench.py --config e2e --steps 30 --warmup 10 --no-cpu > $OUT/slots_e2e_${tag}_$r.json 2>/dev/null || exit $?
  done
done
unset CIO_AMD_LIB
python3 - <<'PY'
import json
for tag in ("s2", "s3", "s4", "s6"):
    for r in (1, 2, 3):
        d = json.loads(open(f"gpurun_out/r03l/slots_e2e_{tag}_{r}.json").read().strip().splitlines()[-1])
        print(tag, r, "staged", d["value"], "registered", d["registered_in_place"]["value"],
              "pinned_h2d", d["breakdown"]["pinned_h2d_GBps"], d["check"])
PY
