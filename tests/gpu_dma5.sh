# LDS-DMA conv on the one-chunk HR shapes (CLIMSR_CONV_DMA_PW=1): conv + bench-shape parity (and EP 1 / 2 on it), then
# the GAN step A/B
set -o pipefail
mkdir -p gpurun_out
T=${1:-d6}
CLIMSR_CONV_DMA_PW=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_bench_shapes.py > gpurun_out/${T}_pytest.log 2>&1 || exit $?
CLIMSR_CONV_DMA=2 timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_conv.py -k lds_dma > gpurun_out/${T}_dma2.log 2>&1 || exit $?
for r in 1 2; do
  CLIMSR_CONV_DMA_PW=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_pw_$r.json 2>> gpurun_out/${T}_bench.err || exit $?
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_nopw_$r.json 2>> gpurun_out/${T}_bench.err || exit $?
done
