# Fused RDB chain check: parity tests, kernel micro-benchmark, pretrain + GAN bench lines.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_generator.py tests/test_gpu_bench_shapes.py -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_chain.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python3 -u tests/perf_conv.py --rdb-only > gpurun_out/perf_chain.log 2>&1 || exit $?
echo "perf ok"
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --median-steps 20 > gpurun_out/bench_chain.json 2> gpurun_out/bench_chain.err || exit $?
echo "bench ok"
