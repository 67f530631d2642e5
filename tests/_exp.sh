set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_generator.py -x -q --timeout 120 --timeout-method thread > gpurun_out/exp_tests.log 2>&1
echo "== PF" > gpurun_out/exp.log
timeout -k 10 100 python tests/perf_conv.py --rdb-only >> gpurun_out/exp.log 2>&1
echo "== NO_PF" >> gpurun_out/exp.log
CLIMSR_NO_FWD_PF=1 timeout -k 10 100 python tests/perf_conv.py --rdb-only >> gpurun_out/exp.log 2>&1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/exp_bench.json 2> gpurun_out/exp_bench.err
