# Round-6 call o: the whole -m gpu suite, smoke, determinism, then same-box A/B against ab/lib_v3.so (the r06_v3
# build) of the 1024-thread BatchNorm partial-sum finish (GAN step) and the overlapped ca_mlp loads (config 5 RCAN),
# alternating.
set -o pipefail
T=${1:-r06o}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/det_check.py new > gpurun_out/${T}_det.json 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-config2 > gpurun_out/${T}_bench_new_$i.json 2> gpurun_out/${T}_bench_new_$i.err || exit $?
  CLIMSR_HIP_LIB=$PWD/ab/lib_v3.so timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-config2 > gpurun_out/${T}_bench_prev_$i.json 2> gpurun_out/${T}_bench_prev_$i.err || exit $?
  timeout -k 10 400 python -u bench.py --mode infer --no-cpu-baseline > gpurun_out/${T}_infer_new_$i.json 2> gpurun_out/${T}_infer_new_$i.err || exit $?
  CLIMSR_HIP_LIB=$PWD/ab/lib_v3.so timeout -k 10 400 python -u bench.py --mode infer --no-cpu-baseline > gpurun_out/${T}_infer_prev_$i.json 2> gpurun_out/${T}_infer_prev_$i.err || exit $?
done
echo done
