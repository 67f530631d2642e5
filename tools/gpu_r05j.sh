# Round 5, call j: 16-B epilogue stores (v_permlane16_swap) in conv_wr, the LDS-DMA convs (stride 1 / 2), the D stem
# and the RDB chain (fragment halves traded by v_permlane16_swap, HBM row stores
# only on the strip's own rows): determinism, the conv / GAN / bench-shape suites, timing vs the previous chain, GAN
# step (alternating).   usage: bash tools/gpu_r05j.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05j}
D=$PWD/climate-super-resolution_amd/csrc/diag
timeout -k 10 240 python -u tools/det_check.py new > gpurun_out/${T}_det.jsonl 2> gpurun_out/${T}_det.err || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_gan.py tests/test_gpu_bench_shapes.py tests/test_gpu_generator.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 120 python -u tools/perf_diag.py new >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_HIP_LIB=$D/chainprev/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py chainprev >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  timeout -k 10 120 python -u tools/perf_wr.py new >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
  CLIMSR_HIP_LIB=$D/chainprev/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_wr.py prev >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
  timeout -k 10 120 python -u tools/perf_s2.py new >> gpurun_out/${T}_s2.jsonl 2>> gpurun_out/${T}_s2.err || exit $?
  CLIMSR_HIP_LIB=$D/chainprev/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_s2.py prev >> gpurun_out/${T}_s2.jsonl 2>> gpurun_out/${T}_s2.err || exit $?
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_new_$i.json 2> gpurun_out/${T}_bench_new_$i.err || exit $?
  CLIMSR_HIP_LIB=$D/chainprev/libclimsr_hip.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_prev_$i.json 2> gpurun_out/${T}_bench_prev_$i.err || exit $?
done
echo done
