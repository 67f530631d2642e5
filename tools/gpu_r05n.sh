# Round 5, call n: RDB conv5 / pull-x on the LDS-DMA conv (diagnostic build dmaep12) and the LDS-DMA wgrad64 with
# an x-fragment lookahead of 3 (w64la3) against this build: kernel timing and the GAN step, alternating.   usage: bash tools/gpu_r05n.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05n}
D=$PWD/climate-super-resolution_amd/csrc/diag
for i in 1 2; do
  timeout -k 10 120 python -u tools/perf_diag.py new >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_HIP_LIB=$D/dmaep12/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py dmaep12 >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_HIP_LIB=$D/w64la3/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py w64la3 >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_new_$i.json 2> gpurun_out/${T}_bench_new_$i.err || exit $?
  CLIMSR_HIP_LIB=$D/dmaep12/libclimsr_hip.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_ep12_$i.json 2> gpurun_out/${T}_bench_ep12_$i.err || exit $?
  CLIMSR_HIP_LIB=$D/w64la3/libclimsr_hip.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_la3_$i.json 2> gpurun_out/${T}_bench_la3_$i.err || exit $?
done
echo done
