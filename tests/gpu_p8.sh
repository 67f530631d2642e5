# GPU check + A/B of the workgroup stagger (CLIMSR_CONV_STAGGER) and a kernel-trace profile of the default build.
# Stops at the first failing / faulting step.
mkdir -p gpurun_out
T=${1:-p8}
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bn_fused.py tests/test_gpu_gan.py \
  tests/test_gpu_plain_d.py > gpurun_out/${T}_pytest.log 2>&1 || exit $?
bash tests/_ab_env.sh $T base CLIMSR_CONV_STAGGER=2 CLIMSR_CONV_STAGGER=3 CLIMSR_CONV_STAGGER=4 || exit $?
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- \
  python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --median-steps 0 --no-config2 > gpurun_out/${T}_prof_bench.json 2> gpurun_out/${T}_prof.err
