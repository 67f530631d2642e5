# GPU check of the LDS-DMA conv: its parity tests + the conv op tests, then A/B timing (perf_diag + GAN step)
set -o pipefail
mkdir -p gpurun_out
T=${1:-d1}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv.py > gpurun_out/${T}_pytest_conv.log 2>&1 || exit $?
bash tests/_ab_env.sh $T CLIMSR_CONV_DMA=0 base
