set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_generator.py tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/exp_tests.log 2>&1
timeout -k 10 100 python tests/perf_conv.py --rdb-only --reps 30 > gpurun_out/exp_rdb.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/exp_bench.json 2> gpurun_out/exp_bench.err
