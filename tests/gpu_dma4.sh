# persistent LDS-DMA conv: conv + fused-BN parity, then perf_diag (persistent / one item per workgroup / old kernel)
# and the GAN step with / without the DMA conv
set -o pipefail
mkdir -p gpurun_out
T=${1:-d4}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_bn_fused.py > gpurun_out/${T}_pytest.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 120 python -u tests/perf_diag.py persist >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_CONV_DMA_PERSIST=0 timeout -k 10 120 python -u tests/perf_diag.py item >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_CONV_DMA=0 timeout -k 10 120 python -u tests/perf_diag.py old >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
done
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_dma_$r.json 2>> gpurun_out/${T}_bench.err || exit $?
  CLIMSR_CONV_DMA=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_old_$r.json 2>> gpurun_out/${T}_bench.err || exit $?
done
