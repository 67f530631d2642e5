# Round 5, call f: rdb5 step-cost attribution -- the product build vs diagnostic builds without the step's DMA (x1),
# residual loads (x2), stores (x3), all three (x4), or MFMAs (x5).   usage: bash tools/gpu_r05f.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05f}
D=$PWD/climate-super-resolution_amd/csrc/diag
for i in 1 2; do
  timeout -k 10 120 python -u tools/perf_diag.py new >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  for v in r5x1 r5x2 r5x3 r5x4 r5x5; do
    CLIMSR_HIP_LIB=$D/$v/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py $v >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  done
done
echo done
