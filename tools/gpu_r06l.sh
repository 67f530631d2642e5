# Round-6 call l: the whole -m gpu suite, smoke, determinism, then the RCAN whole-grid inference line (config 5) of the
# per-wave channel-sum build against ab/lib_base.so (the committed build), alternating.
set -o pipefail
T=${1:-r06l}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/det_check.py new > gpurun_out/${T}_det.json 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --mode infer --no-cpu-baseline > gpurun_out/${T}_infer_new_$i.json 2> gpurun_out/${T}_infer_new_$i.err || exit $?
  CLIMSR_HIP_LIB=$PWD/ab/lib_base.so timeout -k 10 400 python -u bench.py --mode infer --no-cpu-baseline > gpurun_out/${T}_infer_base_$i.json 2> gpurun_out/${T}_infer_base_$i.err || exit $?
done
echo done
