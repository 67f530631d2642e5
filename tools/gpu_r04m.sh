# stride-2 LDS-DMA weight gradient: parity suites touching it, A/B timing against the register-staged kernel
# (diag/w64s2old: -DCLIMSR_W64S2_GLDS=0), then the GAN bench.   usage: bash tools/gpu_r04m.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04m}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_bench_shapes.py tests/test_gpu_gan.py tests/test_gpu_plain_d.py > gpurun_out/${T}_test.log 2>&1 || exit $?
OLD=$PWD/climate-super-resolution_amd/csrc/diag/w64s2old/libclimsr_hip.so
for i in 1 2; do
  timeout -k 10 120 python -u tools/perf_s2.py glds >> gpurun_out/${T}_s2.jsonl 2>> gpurun_out/${T}_s2.err || exit $?
  CLIMSR_HIP_LIB=$OLD timeout -k 10 120 python -u tools/perf_s2.py old >> gpurun_out/${T}_s2.jsonl 2>> gpurun_out/${T}_s2.err || exit $?
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
echo done
