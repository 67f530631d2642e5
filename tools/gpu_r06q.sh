# Round-6 call q: the AdamW tests, the whole -m gpu suite, smoke, then GAN bench lines of the two-group AdamW build
# against ab/lib_v3.so (the r06_v3 build), alternating, same box.
set -o pipefail
T=${1:-r06q}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_adamw.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_adamw.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-config2 > gpurun_out/${T}_bench_new_$i.json 2> gpurun_out/${T}_bench_new_$i.err || exit $?
  CLIMSR_HIP_LIB=$PWD/ab/lib_v3.so timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-config2 > gpurun_out/${T}_bench_prev_$i.json 2> gpurun_out/${T}_bench_prev_$i.err || exit $?
done
echo done
