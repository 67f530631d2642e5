# Round 5, call w: BatchNorm finish kernels at 1024 threads (8 channels x 128 slices, fixed two-level tree) and the BN
# streaming grids at 2048 target workgroups: the BN / D tests, a rocprofv3 kernel-stats pass of a short GAN bench, the
# GAN bench twice.   usage: bash tools/gpu_r05w.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05w}
timeout -k 10 400 python -u -m pytest tests/test_gpu_bn_fused.py tests/test_gpu_conv.py tests/test_gpu_gan.py tests/test_gpu_plain_d.py tests/test_gpu_timed_step.py tests/test_gpu_bench_shapes.py -x -q --timeout 120 --timeout-method thread -m gpu -k "bn or discriminator or timed or plain" > gpurun_out/${T}_tests.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --median-steps 0 --no-config2 --no-cpu-baseline --no-kernel-timing > gpurun_out/${T}_prof.log 2>&1 || exit $?
f=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${T}_kernel_stats.csv; rm -rf gpurun_out/${T}_prof
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_$i.json 2> gpurun_out/${T}_bench_$i.err || exit $?
done
echo done
