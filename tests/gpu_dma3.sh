# LDS-DMA conv: conv + fused-BN parity, then perf_diag under the default build and each diag/*.so (two rounds)
set -o pipefail
mkdir -p gpurun_out
T=${1:-d3}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_bn_fused.py > gpurun_out/${T}_pytest.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 120 python -u tests/perf_diag.py dma >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  for L in diag/*.so; do
    CLIMSR_HIP_LIB=$PWD/$L timeout -k 10 120 python -u tests/perf_diag.py $(basename $L) >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  done
done
