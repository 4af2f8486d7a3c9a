set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 && tail -3 $O/pytest_gpu.txt &&
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err && echo default-ok &&
CIO_BENCH_REHEARSE=1 timeout -k 10 700 python bench.py --gpus 2 > $O/bench_rehearse_n2.json 2> $O/bench_rehearse_n2.err && echo n2-ok &&
{ CIO_BENCH_SHARE_DEVICES=1 timeout -k 10 300 python bench.py --gpus 2 --no-extra --steps 20 --warmup 5 > $O/bench_share_n2.json 2> $O/bench_share_n2.err; echo "share rc=$?" | tee $O/share_rc.txt; }
