# Round 5, first call: the GPU suite + smoke on the merged round-4 variants (branch wip-r04-unvalidated) and the
# stride-2 DMA wait fix, then same-box alternating A/B of each variant against its predecessor (csrc/diag/*, built by
# tools/build_r05_ab.sh) and of the whole build against main's round-4 conv sources (diag/main).
#   usage: bash tools/gpu_r05a.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05a}
D=$PWD/climate-super-resolution_amd/csrc/diag
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 120 python -u tools/perf_wr.py new >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
  CLIMSR_HIP_LIB=$D/wrold/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_wr.py old >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
  CLIMSR_HIP_LIB=$D/wrmid/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_wr.py mid >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
  timeout -k 10 120 python -u tools/perf_s2.py glds >> gpurun_out/${T}_s2.jsonl 2>> gpurun_out/${T}_s2.err || exit $?
  CLIMSR_HIP_LIB=$D/w64s2old/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_s2.py old >> gpurun_out/${T}_s2.jsonl 2>> gpurun_out/${T}_s2.err || exit $?
  timeout -k 10 120 python -u tools/perf_diag.py dma_act1 >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_HIP_LIB=$D/dmaold/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py dma_old >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_HIP_LIB=$D/dmasp2/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py dma_sp2 >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  CLIMSR_HIP_LIB=$D/dmasp3/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py dma_sp3 >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
  timeout -k 10 120 python -u tools/perf_co1m.py new >> gpurun_out/${T}_co1m.jsonl 2>> gpurun_out/${T}_co1m.err || exit $?
  CLIMSR_HIP_LIB=$D/main/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_co1m.py main >> gpurun_out/${T}_co1m.jsonl 2>> gpurun_out/${T}_co1m.err || exit $?
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_new_$i.json 2> gpurun_out/${T}_bench_new_$i.err || exit $?
  CLIMSR_HIP_LIB=$D/main/libclimsr_hip.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_main_$i.json 2> gpurun_out/${T}_bench_main_$i.err || exit $?
done
timeout -k 10 300 python -u bench.py --mode infer --model rcan --no-cpu-baseline > gpurun_out/${T}_rcan_new.json 2> gpurun_out/${T}_rcan_new.err || exit $?
CLIMSR_HIP_LIB=$D/main/libclimsr_hip.so timeout -k 10 300 python -u bench.py --mode infer --model rcan --no-cpu-baseline > gpurun_out/${T}_rcan_main.json 2> gpurun_out/${T}_rcan_main.err || exit $?
echo done
