# Round 5, call g: rdb5 with 16-B residual loads / stores (fragment halves traded by v_permlane16_swap), conv_wr with
# the footprint DMA back at the tile start: determinism, parity, stamps, timing vs main and the wrmid build.
#   usage: bash tools/gpu_r05g.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05g}
D=$PWD/climate-super-resolution_amd/csrc/diag
timeout -k 10 240 python -u tools/det_check.py new > gpurun_out/${T}_det.jsonl 2> gpurun_out/${T}_det.err || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_gan.py -q --timeout 120 --timeout-method thread > gpurun_out/${T}_conv.log 2>&1 || exit $?
CLIMSR_HIP_LIB=$D/r5stamp/libclimsr_hip.so timeout -k 10 120 python -u tools/stamp_r5.py stamp > gpurun_out/${T}_stamp.jsonl 2> gpurun_out/${T}_stamp.err || exit $?
for i in 1 2; do
  timeout -k 10 120 python -u tools/perf_diag.py new >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_HIP_LIB=$D/main/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py main >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  timeout -k 10 120 python -u tools/perf_wr.py new >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
  CLIMSR_HIP_LIB=$D/wrmid/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_wr.py wrmid >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
done
echo done
