# Fused RDB chain: parity + kernel micro-benchmark only.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_conv.py -k "chain" -m gpu -v -s --timeout 150 --timeout-method thread > gpurun_out/pytest_chain2.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python3 -u tests/perf_conv.py --rdb-only > gpurun_out/perf_chain2.log 2>&1 || exit $?
echo "perf ok"
