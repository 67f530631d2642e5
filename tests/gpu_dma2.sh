# LDS-DMA conv iteration: parity of the conv op tests, then perf_diag under: old kernel, DMA kernel, diagnostic libs
set -o pipefail
mkdir -p gpurun_out
T=${1:-d2}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py > gpurun_out/${T}_pytest_conv.log 2>&1 || exit $?
for r in 1 2; do
  CLIMSR_CONV_DMA=0 timeout -k 10 120 python -u tests/perf_diag.py old >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  timeout -k 10 120 python -u tests/perf_diag.py dma >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  for L in diag/*.so; do
    CLIMSR_HIP_LIB=$PWD/$L timeout -k 10 120 python -u tests/perf_diag.py $(basename $L) >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  done
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2>> gpurun_out/${T}_bench.err || exit $?
