#!/bin/bash
# cfg4 (8192 x 4 MiB at N = 1) standalone, in the default line, and in the
# default line without its host-memory legs.  Usage: bash profiles/r04/scripts/cfg4_order.sh TAG
set -u
D=gpurun_out/$1; mkdir -p $D
timeout -k 10 200 python bench.py --config cfg4 --steps 20 --warmup 5 --no-cpu > $D/cfg4_alone.json 2> $D/cfg4_alone.err || exit $?
timeout -k 10 400 python bench.py > $D/default.json 2> $D/default.err || exit $?
CIO_BENCH_LEGS=cfg3,sha1 timeout -k 10 400 python bench.py > $D/default_nohost.json 2> $D/default_nohost.err || exit $?
timeout -k 10 200 python bench.py --config cfg4 --steps 20 --warmup 5 --no-cpu > $D/cfg4_alone2.json 2> $D/cfg4_alone2.err || exit $?
python3 - "$D" <<'PY'
import json, sys
d = sys.argv[1]
for f in ("cfg4_alone", "default", "default_nohost", "cfg4_alone2"):
    a = json.load(open(f"{d}/{f}.json"))
    c = a if f.startswith("cfg4") else a["other_chunk_sizes"]["cfg4"]
    print(f"{f:>16}: cfg4 frac {c['roofline']['frac']}  kernel_ms {c['roofline']['kernel_ms_mean']}")
PY
