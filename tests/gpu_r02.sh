# Round-2 GPU check: -m gpu tests, the default bench line, a rocprofv3 kernel-stats pass of the GAN step.
# Stops at the first step that crashes / times out (anything but pass or plain test failures).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
echo "bench ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gan -o run -- python3 -u bench.py --no-cpu-baseline --no-config2 --no-kernel-timing --steps 20 --warmup 5 --median-steps 0 > gpurun_out/prof_gan.json 2> gpurun_out/prof_gan.err || exit $?
echo "prof ok"
