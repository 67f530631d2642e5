# Round 5, call o: weight-gradient reductions on a side stream (ops.Workspace): the GAN / generator / bench-shape /
# timed-step / DDP / config suites, and the GAN step against the same build with the reductions in stream order.
#   usage: bash tools/gpu_r05o.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05o}
timeout -k 10 900 python -u -m pytest tests/test_gpu_gan.py tests/test_gpu_generator.py tests/test_gpu_bench_shapes.py tests/test_gpu_timed_step.py tests/test_gpu_ddp.py tests/test_gpu_configs.py tests/test_gpu_plain_d.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_side_$i.json 2> gpurun_out/${T}_bench_side_$i.err || exit $?
  timeout -k 10 300 python -u tools/bench_serial_reduce.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_serial_$i.json 2> gpurun_out/${T}_bench_serial_$i.err || exit $?
done
echo done
