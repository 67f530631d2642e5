# Round-6 call j: the whole -m gpu suite, smoke, determinism, the wgrad64 A/B (bias sums on one wave per quad vs
# ab/lib_prev.so, the previous commit's weight-gradient TU), alternating, and the GAN bench.
set -o pipefail
T=${1:-r06j}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/det_check.py new > gpurun_out/${T}_det.json 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python -u tools/perf_wgrad64.py new >> gpurun_out/${T}_wg.json 2>&1 || exit $?
  CLIMSR_HIP_LIB=$PWD/ab/lib_prev.so timeout -k 10 200 python -u tools/perf_wgrad64.py prev >> gpurun_out/${T}_wg.json 2>&1 || exit $?
done
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_gan_bench.json 2> gpurun_out/${T}_gan_bench.err || exit $?
echo done
