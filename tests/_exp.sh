set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/exp_tests.log 2>&1
CLIMSR_BENCH_DETAIL=1 timeout -k 10 300 python bench.py --mode gan --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/exp_gan.json 2> gpurun_out/exp_gan.err
