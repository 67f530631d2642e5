# Round 5, call d: rdb5 time breakdown (stamp build), conv GPU tests (+ fused conv/ReLU/max-pool), stem and pool
# fusion A/B, the variant A/B that call c could not load, and the GAN step vs main (alternating).
#   usage: bash tools/gpu_r05d.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05d}
D=$PWD/climate-super-resolution_amd/csrc/diag
CLIMSR_HIP_LIB=$D/r5stamp/libclimsr_hip.so timeout -k 10 120 python -u tools/stamp_r5.py stamp > gpurun_out/${T}_stamp.jsonl 2> gpurun_out/${T}_stamp.err || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_gan.py tests/test_gpu_bench_shapes.py -q --timeout 120 --timeout-method thread > gpurun_out/${T}_conv.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/perf_stem.py new > gpurun_out/${T}_stem.jsonl 2> gpurun_out/${T}_stem.err || exit $?
timeout -k 10 120 python -u tools/perf_diag.py new >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
for v in main r5v1 dmasp2 dmasp3 dmaold; do
  CLIMSR_HIP_LIB=$D/$v/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_diag.py $v >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
done
timeout -k 10 120 python -u tools/perf_wr.py new >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
for v in wrold wrmid; do
  CLIMSR_HIP_LIB=$D/$v/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_wr.py $v >> gpurun_out/${T}_wr.jsonl 2>> gpurun_out/${T}_wr.err || exit $?
done
timeout -k 10 120 python -u tools/perf_s2.py glds >> gpurun_out/${T}_s2.jsonl 2>> gpurun_out/${T}_s2.err || exit $?
CLIMSR_HIP_LIB=$D/w64s2old/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_s2.py old >> gpurun_out/${T}_s2.jsonl 2>> gpurun_out/${T}_s2.err || exit $?
timeout -k 10 120 python -u tools/perf_co1m.py new >> gpurun_out/${T}_co1m.jsonl 2>> gpurun_out/${T}_co1m.err || exit $?
CLIMSR_HIP_LIB=$D/main/libclimsr_hip.so timeout -k 10 120 python -u tools/perf_co1m.py main >> gpurun_out/${T}_co1m.jsonl 2>> gpurun_out/${T}_co1m.err || exit $?
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_new_$i.json 2> gpurun_out/${T}_bench_new_$i.err || exit $?
  CLIMSR_HIP_LIB=$D/main/libclimsr_hip.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_main_$i.json 2> gpurun_out/${T}_bench_main_$i.err || exit $?
done
echo done
