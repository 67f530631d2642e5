# Round 4: chain prefetch / srcnn tail / RCAN fold -- parity suites, GAN bench, config-5 inference
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04g}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv.py > gpurun_out/${T}_conv.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_generator.py tests/test_gpu_bench_shapes.py tests/test_gpu_configs.py tests/test_gpu_rcan.py > gpurun_out/${T}_g.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
timeout -k 10 300 python -u bench.py --mode infer --model esrgan --no-cpu-baseline > gpurun_out/${T}_infer_esrgan.json 2> gpurun_out/${T}_infer.err || exit $?
timeout -k 10 300 python -u bench.py --mode infer --model rcan --no-cpu-baseline > gpurun_out/${T}_infer_rcan.json 2>> gpurun_out/${T}_infer.err || exit $?
bash tools/gpu_chain_prof.sh ${T}_ch || exit $?
