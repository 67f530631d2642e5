# Round-6 GPU call: a named subset of the -m gpu suite (pytest -k / file list in $TESTS), then optional bench lines.
# usage: TESTS="tests/test_gpu_rcan.py" BENCH="gan infer_rcan" bash tools/gpu_r06.sh <tag>
set -o pipefail
T=${1:-r06a}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread ${KEXPR:+-k "$KEXPR"} > gpurun_out/${T}_pytest.log 2>&1 || exit $?
fi
for b in $BENCH; do
  case $b in
    gan) timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_gan_bench.json 2> gpurun_out/${T}_gan_bench.err || exit $? ;;
    infer_rcan) timeout -k 10 300 python -u bench.py --mode infer --model rcan --no-cpu-baseline > gpurun_out/${T}_infer_rcan.json 2> gpurun_out/${T}_infer_rcan.err || exit $? ;;
    *) echo "unknown bench $b"; exit 2 ;;
  esac
done
echo done
