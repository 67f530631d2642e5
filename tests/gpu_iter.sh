# Iteration check: full -m gpu suite, then the bench line with the per-tag kernel breakdown.
T=${1:-i1}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 540 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
grep -E "FAILED|passed|failed" gpurun_out/${T}_pytest.log | tail -8
CLIMSR_BENCH_DETAIL=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
echo "bench ok"
