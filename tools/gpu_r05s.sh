# Round 5, call s: two-phase BatchNorm finishes (bn_finish2_kernel), the 16 B adaptive-pool tile kernels and RCAN's
# one-launch channel attention (ca_parts_mlp_kernel): their
# tests, the whole -m gpu suite, a rocprofv3 kernel-stats pass of a short GAN bench, then the GAN and RCAN benches.
#   usage: bash tools/gpu_r05s.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05s}
timeout -k 10 300 python -u -m pytest tests/test_gpu_bn_fused.py tests/test_gpu_conv.py tests/test_gpu_gan.py tests/test_gpu_rcan.py -x -v --timeout 120 --timeout-method thread -m gpu -k "bn or discriminator or attention or rcan" > gpurun_out/${T}_bn_tests.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/${T}_pytest_gpu.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --median-steps 0 --no-config2 --no-cpu-baseline --no-kernel-timing > gpurun_out/${T}_prof.log 2>&1 || exit $?
f=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${T}_kernel_stats.csv; rm -rf gpurun_out/${T}_prof
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_$i.json 2> gpurun_out/${T}_bench_$i.err || exit $?
  timeout -k 10 300 python -u bench.py --mode infer --model rcan --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/${T}_rcan_$i.json 2> gpurun_out/${T}_rcan_$i.err || exit $?
done
echo done
