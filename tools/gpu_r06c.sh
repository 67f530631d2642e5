# Round-6 call c: the whole -m gpu suite (loss-scalar deviations printed: -s on the step tests), smoke, the GAN bench,
# run-to-run determinism, and the D stem A/B against ab/libclimsr_hip_old.so (round 5's kernels).
set -o pipefail
T=${1:-r06d}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_gan.py tests/test_gpu_bench_shapes.py tests/test_gpu_generator.py tests/test_gpu_configs.py tests/test_gpu_rcan.py -m gpu -x -q -s --timeout 300 --timeout-method thread -k "loss or step or golden or training or config or perceptual" > gpurun_out/${T}_loss_scalars.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_gan_bench.json 2> gpurun_out/${T}_gan_bench.err || exit $?
timeout -k 10 200 python -u tools/det_check.py new > gpurun_out/${T}_det.json 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python -u tools/perf_dstem.py new >> gpurun_out/${T}_dstem.json 2>&1 || exit $?
  CLIMSR_HIP_LIB=$PWD/ab/libclimsr_hip_old.so timeout -k 10 200 python -u tools/perf_dstem.py old >> gpurun_out/${T}_dstem.json 2>&1 || exit $?
done
echo done
