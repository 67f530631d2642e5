# Round-6 call k: the whole -m gpu suite, smoke, determinism, the persistent BatchNorm-partials conv A/B against
# ab/lib_prev.so (the previous commit's build), alternating, and GAN bench lines of both builds.
set -o pipefail
T=${1:-r06k}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/det_check.py new > gpurun_out/${T}_det.json 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python -u tools/perf_dbn.py new >> gpurun_out/${T}_dbn.json 2>&1 || exit $?
  CLIMSR_HIP_LIB=$PWD/ab/lib_prev.so timeout -k 10 200 python -u tools/perf_dbn.py prev >> gpurun_out/${T}_dbn.json 2>&1 || exit $?
done
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-config2 > gpurun_out/${T}_bench_new_$i.json 2> gpurun_out/${T}_bench_new_$i.err || exit $?
  CLIMSR_HIP_LIB=$PWD/ab/lib_prev.so timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-config2 > gpurun_out/${T}_bench_prev_$i.json 2> gpurun_out/${T}_bench_prev_$i.err || exit $?
done
echo done
