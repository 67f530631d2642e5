# Round 5, call h: chain step-cost attribution (no step DMA / no HBM row stores / no MFMAs), conv5 + pull-x back on the
# implicit GEMM (determinism, parity), GAN step with vs without the rdb5 route (alternating).
#   usage: bash tools/gpu_r05h.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05h}
D=$PWD/climate-super-resolution_amd/csrc/diag
timeout -k 10 240 python -u tools/det_check.py new > gpurun_out/${T}_det.jsonl 2> gpurun_out/${T}_det.err || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -q -k "rdb5 or chain" --timeout 120 --timeout-method thread > gpurun_out/${T}_conv.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 120 python -u tools/perf_diag.py new >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  for v in rrx1 rrx3 rrx5; do
    CLIMSR_HIP_LIB=$D/$v/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py $v >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  done
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_new_$i.json 2> gpurun_out/${T}_bench_new_$i.err || exit $?
  CLIMSR_HIP_LIB=$D/rdb5on/libclimsr_hip.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_rdb5_$i.json 2> gpurun_out/${T}_bench_rdb5_$i.err || exit $?
done
echo done
