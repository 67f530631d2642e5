# A/B timing of library variants in one GPU call: tools/perf_diag.py under each CLIMSR_HIP_LIB (args: tag variant...)
set -o pipefail
mkdir -p gpurun_out
T=$1; shift
for v in "$@"; do
  if [ $v = base ]; then lib=climate-super-resolution_amd/csrc/libclimsr_hip.so; else lib=climate-super-resolution_amd/csrc/diag/$v/libclimsr_hip.so; fi
  CLIMSR_HIP_LIB=$PWD/$lib timeout -k 10 120 python -u tools/perf_diag.py $v >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
done
