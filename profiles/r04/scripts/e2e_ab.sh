set -u
mkdir -p gpurun_out
for r in 1 2 3; do
  CIO_AMD_LIB=chunkio_amd/lib/ab/prev_pipe.so timeout -k 10 120 python bench.py --config e2e --steps 30 --warmup 10 --no-cpu > gpurun_out/e2e_prev_$r.json 2>/dev/null || exit $?
  timeout -k 10 120 python bench.py --config e2e --steps 30 --warmup 10 --no-cpu > gpurun_out/e2e_new_$r.json 2>/dev/null || exit $?
done
python3 - <<'PY'
import json
for tag in ("prev","new"):
    for r in (1,2,3):
        d=json.load(open(f"gpurun_out/e2e_{tag}_{r}.json"))
        print(tag, r, "staged", d["value"], "registered", d["registered_in_place"]["value"], d["check"])
PY
