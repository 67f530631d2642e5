# Round 5, call c: determinism (this build, the previous rdb5 in diag/r5v1), the conv GPU tests, RDB kernel timing vs
# main's round-4 build and r5v1, the round-4 variant A/B that never ran, and the GAN step vs main (alternating).
#   usage: bash tools/gpu_r05c.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05c}
D=$PWD/climate-super-resolution_amd/csrc/diag
timeout -k 10 240 python -u tools/det_check.py new > gpurun_out/${T}_det.jsonl 2> gpurun_out/${T}_det.err || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_gan.py tests/test_gpu_bench_shapes.py -q --timeout 120 --timeout-method thread > gpurun_out/${T}_conv.log 2>&1
for i in 1 2; do
  timeout -k 10 120 python -u tools/perf_diag.py new >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_HIP_LIB=$D/main/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py main >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_HIP_LIB=$D/r5v1/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py r5v1 >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_HIP_LIB=$D/dmasp2/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py dma_sp2 >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_HIP_LIB=$D/dmasp3/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py dma_sp3 >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_HIP_LIB=$D/dmaold/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py dma_old >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  timeout -k 10 120 python -u tools/perf_wr.py new >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
  CLIMSR_HIP_LIB=$D/wrold/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_wr.py old >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
  CLIMSR_HIP_LIB=$D/wrmid/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_wr.py mid >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
  timeout -k 10 120 python -u tools/perf_s2.py glds >> gpurun_out/${T}_s2.jsonl 2>> gpurun_out/${T}_s2.err || exit $?
  CLIMSR_HIP_LIB=$D/w64s2old/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_s2.py old >> gpurun_out/${T}_s2.jsonl 2>> gpurun_out/${T}_s2.err || exit $?
  timeout -k 10 120 python -u tools/perf_co1m.py new >> gpurun_out/${T}_co1m.jsonl 2>> gpurun_out/${T}_co1m.err || exit $?
  CLIMSR_HIP_LIB=$D/main/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_co1m.py main >> gpurun_out/${T}_co1m.jsonl 2>> gpurun_out/${T}_co1m.err || exit $?
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_new_$i.json 2> gpurun_out/${T}_bench_new_$i.err || exit $?
  CLIMSR_HIP_LIB=$D/main/libclimsr_hip.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_main_$i.json 2> gpurun_out/${T}_bench_main_$i.err || exit $?
done
echo done
