# DMA-conv direct epilogues (EP 3 / 6 / 8 / 9): parity suites touching the D / VGG convs, timing, GAN bench
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04h}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_bn_fused.py tests/test_gpu_plain_d.py tests/test_gpu_gan.py tests/test_gpu_bench_shapes.py > gpurun_out/${T}_test.log 2>&1 || exit $?
timeout -k 10 120 python -u tools/perf_diag.py direct > gpurun_out/${T}_diag.jsonl 2> gpurun_out/${T}_diag.err || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
