# Per-tag kernel breakdown of the GAN step (bench.py's eager HIP-event timer) + selected GPU tests.
# usage: bash tests/gpu_detail.sh <tag> [pytest node ids...]
T=${1:-d1}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -v -s --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi
fi
CLIMSR_BENCH_DETAIL=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-config2 --steps 5 --warmup 2 --median-steps 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
echo "bench ok"
