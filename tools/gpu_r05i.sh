# Round 5, call i: conv_wr with the weights staged through LDS once per workgroup (parity: conv / RCAN / GAN suites;
# timing vs the previous build: conv_wr shapes, RCAN whole grid), chain step-cost attribution, and the GAN step:
# this build vs the previous one (conv_wr) vs the previous one with the rdb5 route (alternating).
#   usage: bash tools/gpu_r05i.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05i}
D=$PWD/climate-super-resolution_amd/csrc/diag
timeout -k 10 900 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_rcan.py tests/test_gpu_configs.py tests/test_gpu_gan.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit $?
timeout -k 10 240 python -u tools/det_check.py new > gpurun_out/${T}_det.jsonl 2> gpurun_out/${T}_det.err || exit $?
for i in 1 2; do
  timeout -k 10 120 python -u tools/perf_wr.py new >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
  CLIMSR_HIP_LIB=$D/wrprev/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_wr.py wrprev >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
  timeout -k 10 300 python -u bench.py --mode infer --model rcan --no-cpu-baseline > gpurun_out/${T}_rcan_new_$i.json 2> gpurun_out/${T}_rcan_new_$i.err || exit $?
  CLIMSR_HIP_LIB=$D/wrprev/libclimsr_hip.so timeout -k 10 300 python -u bench.py --mode infer --model rcan --no-cpu-baseline > gpurun_out/${T}_rcan_prev_$i.json 2> gpurun_out/${T}_rcan_prev_$i.err || exit $?
done
timeout -k 10 120 python -u tools/perf_diag.py new >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
for v in rrx1 rrx3 rrx5; do
  CLIMSR_HIP_LIB=$D/$v/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py $v >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_new_$i.json 2> gpurun_out/${T}_bench_new_$i.err || exit $?
  CLIMSR_HIP_LIB=$D/wrprev/libclimsr_hip.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_prev_$i.json 2> gpurun_out/${T}_bench_prev_$i.err || exit $?
  CLIMSR_HIP_LIB=$D/rdb5on/libclimsr_hip.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_rdb5_$i.json 2> gpurun_out/${T}_bench_rdb5_$i.err || exit $?
done
echo done
