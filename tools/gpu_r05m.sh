# Round 5, call m: the RDB chain's weights staged through LDS once per workgroup: determinism, suites, chain timing
# and the GAN step against the profiled build (diag/v1, alternating).   usage: bash tools/gpu_r05m.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05m}
D=$PWD/climate-super-resolution_amd/csrc/diag
timeout -k 10 240 python -u tools/det_check.py new > gpurun_out/${T}_det.jsonl 2> gpurun_out/${T}_det.err || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_gan.py tests/test_gpu_bench_shapes.py tests/test_gpu_generator.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 120 python -u tools/perf_diag.py new >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_HIP_LIB=$D/v1/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py v1 >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_new_$i.json 2> gpurun_out/${T}_bench_new_$i.err || exit $?
  CLIMSR_HIP_LIB=$D/v1/libclimsr_hip.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_v1_$i.json 2> gpurun_out/${T}_bench_v1_$i.err || exit $?
done
echo done
