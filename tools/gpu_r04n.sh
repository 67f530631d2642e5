# conv_wr with the activation as a template parameter and one-add DMA offsets for interior tiles: the conv / RCAN
# parity suites, LDS-DMA conv with the epilogue activation resolved per item (diag/dmaold: per element), A/B timing against the previous conv_wr (diag/wrold; diag/wrmid: templated, DMA issued at the tile's start), stride-2 wgrad A/B (diag/w64s2old), GAN bench.
#   usage: bash tools/gpu_r04n.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04n}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_rcan.py tests/test_gpu_bench_shapes.py tests/test_gpu_gan.py > gpurun_out/${T}_test.log 2>&1 || exit $?
D=$PWD/climate-super-resolution_amd/csrc/diag
for i in 1 2; do
  timeout -k 10 120 python -u tools/perf_wr.py new >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
  CLIMSR_HIP_LIB=$D/wrold/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_wr.py old >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
  CLIMSR_HIP_LIB=$D/wrmid/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_wr.py mid >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
  timeout -k 10 120 python -u tools/perf_s2.py glds >> gpurun_out/${T}_s2.jsonl 2>> gpurun_out/${T}_s2.err || exit $?
  CLIMSR_HIP_LIB=$D/w64s2old/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_s2.py old >> gpurun_out/${T}_s2.jsonl 2>> gpurun_out/${T}_s2.err || exit $?
  timeout -k 10 120 python -u tools/perf_diag.py dma_act1 >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_HIP_LIB=$D/dmaold/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py dma_old >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
timeout -k 10 300 python -u bench.py --mode infer --model rcan --no-cpu-baseline > gpurun_out/${T}_rcan.json 2> gpurun_out/${T}_rcan.err || exit $?
echo done
