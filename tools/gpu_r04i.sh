# RCAN with bf16 RCAB outputs (conv_wr EP 4 + bf16 scale-add): parity, config-5 RCAN timing; SRCNN / reduce changes
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04i}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_rcan.py tests/test_gpu_generator.py > gpurun_out/${T}_test.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_configs.py -k "config5" > gpurun_out/${T}_cfg5.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --mode infer --model rcan --no-cpu-baseline > gpurun_out/${T}_infer_rcan.json 2> gpurun_out/${T}_infer.err || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
