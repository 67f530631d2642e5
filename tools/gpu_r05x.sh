# Round 5, call x: the split-K weight-gradient reduce in its 16 B quad form (bit-identical to the scalar form): the reduce
# test, the conv / GAN / timed-step tests, a rocprofv3 kernel-stats pass of a short GAN bench, the GAN bench twice.
#   usage: bash tools/gpu_r05x.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05x}
timeout -k 10 500 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_gan.py tests/test_gpu_timed_step.py tests/test_gpu_bench_shapes.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/${T}_tests.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --median-steps 0 --no-config2 --no-cpu-baseline --no-kernel-timing > gpurun_out/${T}_prof.log 2>&1 || exit $?
f=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${T}_kernel_stats.csv; rm -rf gpurun_out/${T}_prof
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_$i.json 2> gpurun_out/${T}_bench_$i.err || exit $?
done
echo done
