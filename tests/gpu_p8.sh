# GPU check (D / conv parity tests, stopping at the first failing or faulting step) + env A/B of the given settings
# + a kernel-trace profile of the default build.   bash tests/gpu_p8.sh <tag> <setting>...
mkdir -p gpurun_out
T=${1:-p8}; shift
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bn_fused.py tests/test_gpu_conv.py \
  tests/test_gpu_gan.py tests/test_gpu_plain_d.py > gpurun_out/${T}_pytest.log 2>&1 || exit $?
bash tests/_ab_env.sh $T base "$@" || exit $?
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- \
  python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --median-steps 0 --no-config2 > gpurun_out/${T}_prof_bench.json 2> gpurun_out/${T}_prof.err
