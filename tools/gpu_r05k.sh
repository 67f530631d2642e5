# Round 5, call k: the stride-2 LDS-DMA conv's even/odd footprint columns (conflict-free reads) and the pooled
# epilogues' halved store count: determinism, suites, A/B against the profiled build (diag/v1), GAN step (alternating).
#   usage: bash tools/gpu_r05k.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05k}
D=$PWD/climate-super-resolution_amd/csrc/diag
timeout -k 10 240 python -u tools/det_check.py new > gpurun_out/${T}_det.jsonl 2> gpurun_out/${T}_det.err || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_gan.py tests/test_gpu_bench_shapes.py tests/test_gpu_bn_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 120 python -u tools/perf_s2.py new >> gpurun_out/${T}_s2.jsonl 2>> gpurun_out/${T}_s2.err || exit $?
  CLIMSR_HIP_LIB=$D/v1/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_s2.py v1 >> gpurun_out/${T}_s2.jsonl 2>> gpurun_out/${T}_s2.err || exit $?
  timeout -k 10 120 python -u tools/perf_vgg_pool.py new >> gpurun_out/${T}_pool.jsonl 2>> gpurun_out/${T}_pool.err || exit $?
  CLIMSR_HIP_LIB=$D/v1/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_vgg_pool.py v1 >> gpurun_out/${T}_pool.jsonl 2>> gpurun_out/${T}_pool.err || exit $?
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_new_$i.json 2> gpurun_out/${T}_bench_new_$i.err || exit $?
  CLIMSR_HIP_LIB=$D/v1/libclimsr_hip.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_v1_$i.json 2> gpurun_out/${T}_bench_v1_$i.err || exit $?
done
echo done
