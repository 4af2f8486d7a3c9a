#!/bin/bash
# SHA-1 per-batch workgroup geometry: the SHA-1 GPU tests under the automatic
# choice and each forced geometry, the product against the c8/g8 A/B build,
# and the bench's SHA-1 line.
set -u
OUT=gpurun_out/${1:-r03zv}; mkdir -p $OUT; export TMPDIR=/tmp
for g in auto 8 16 32; do
  if [ $g = auto ]; then E=""; else E="CIO_SHA1_CHUNKS_PER_WG=$g"; fi
  env $E timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_sha1.py > $OUT/pytest_sha1_$g.txt 2>&1 || { tail -20 $OUT/pytest_sha1_$g.txt; exit 1; }
  echo "[$g] $(tail -1 $OUT/pytest_sha1_$g.txt)"
done
timeout -k 10 300 python tools/sha1_ab.py --libs chunkio_amd/lib/libchunkio_amd.so,chunkio_amd/lib/ab/sha1_c8g8.so --rounds 5 --iters 10 > $OUT/ab_sha1_geom.txt 2>&1 || { tail -20 $OUT/ab_sha1_geom.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_sha1_geom.txt | tail -3
timeout -k 10 300 python bench.py --config sha1 --steps 10 --warmup 2 --no-cpu > $OUT/bench_sha1.json 2> $OUT/bench_sha1.err || { tail -5 $OUT/bench_sha1.err; exit 1; }
python -c "import json; l=json.loads(open('$OUT/bench_sha1.json').read().strip().splitlines()[-1]); print('bench sha1', l['value'], l['ms_per_step'], l['roofline'].get('frac_of_issue_floor'))"
