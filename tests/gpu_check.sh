# GPU check: new parity tests (stop at the first failure; nothing else runs after one), then A/B timing
mkdir -p gpurun_out
T=${1:-p7}
timeout -k 10 700 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bn_fused.py tests/test_gpu_conv.py \
  tests/test_gpu_bench_shapes.py > gpurun_out/${T}_pytest_a.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_generator.py tests/test_gpu_gan.py \
  tests/test_gpu_plain_d.py tests/test_gpu_ddp.py tests/test_gpu_timed_step.py > gpurun_out/${T}_pytest_b.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -v --timeout 500 --timeout-method thread tests/test_gpu_configs.py::test_config1_trainer_steps_vs_golden \
  > gpurun_out/${T}_pytest_c.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tests/_ab_env.sh $T base CLIMSR_W64_GLDS=0
