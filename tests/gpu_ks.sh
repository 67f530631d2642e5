# GPU check of the K-split GEO-1 conv (CLIMSR_CONV_KS=1): parity tests that dispatch it (stop at the first failing
# or faulting step), then A/B timing against the one-round kernel.
mkdir -p gpurun_out
T=${1:-ks1}
CLIMSR_CONV_KS=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv.py \
  tests/test_gpu_bn_fused.py tests/test_gpu_bench_shapes.py > gpurun_out/${T}_pytest_a.log 2>&1 || exit $?
CLIMSR_CONV_KS=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_gan.py \
  tests/test_gpu_generator.py tests/test_gpu_plain_d.py > gpurun_out/${T}_pytest_b.log 2>&1 || exit $?
bash tests/_ab_env.sh $T base CLIMSR_CONV_KS=1
