# Round 5, call t: RCAN channel attention (call t: one-launch ca_parts_mlp_kernel; call u: ca_mlp_kernel with staged weights) and the 16 B
# adaptive-pool tile kernels: their tests, a rocprofv3 kernel-stats pass of the RCAN whole-grid bench, then the RCAN
# and GAN benches.   usage: bash tools/gpu_r05t.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05t}
timeout -k 10 300 python -u -m pytest tests/test_gpu_rcan.py tests/test_gpu_gan.py tests/test_gpu_bn_fused.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/${T}_tests.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 bench.py --mode infer --model rcan --steps 3 --warmup 1 --median-steps 0 --no-cpu-baseline --no-kernel-timing > gpurun_out/${T}_prof.log 2>&1 || exit $?
f=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${T}_rcan_kernel_stats.csv; rm -rf gpurun_out/${T}_prof
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --mode infer --model rcan --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/${T}_rcan_$i.json 2> gpurun_out/${T}_rcan_$i.err || exit $?
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
echo done
