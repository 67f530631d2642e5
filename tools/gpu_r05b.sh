# Round 5, call b: run-to-run determinism of the hot kernels (tools/det_check.py) on this build and on main's round-4
# conv sources (diag/main), the conv GPU tests, then timing of the RDB kernels and the GAN step against diag/main.
#   usage: bash tools/gpu_r05b.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05b}
D=$PWD/climate-super-resolution_amd/csrc/diag
timeout -k 10 240 python -u tools/det_check.py new > gpurun_out/${T}_det.jsonl 2> gpurun_out/${T}_det.err || exit $?
CLIMSR_HIP_LIB=$D/main/libclimsr_hip.so timeout -k 10 240 python -u tools/det_check.py main >> gpurun_out/${T}_det.jsonl 2>> gpurun_out/${T}_det.err || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -q --timeout 120 --timeout-method thread > gpurun_out/${T}_conv.log 2>&1
for i in 1 2; do
  timeout -k 10 120 python -u tools/perf_diag.py new >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_HIP_LIB=$D/main/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py main >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
done
echo done
