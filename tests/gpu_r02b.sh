mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_shapes.py tests/test_gpu_gan.py tests/test_gpu_conv.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_b.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --no-config2 > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || exit $?
echo "bench ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gan_b -o run -- python3 -u bench.py --no-cpu-baseline --no-config2 --no-kernel-timing --steps 20 --warmup 5 --median-steps 0 > gpurun_out/prof_gan_b.json 2> gpurun_out/prof_gan_b.err || exit $?
echo "prof ok"
