# Round 5, call q: fc.0 microbenchmark (fragment-order forward / data gradient, AdamW fragment-order variants, merged
# weight gradient), the fc.0 / DDP / timed-step GPU tests.   usage: bash tools/gpu_r05q.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05q}
timeout -k 10 180 python -u tools/bench_linear_fc0.py > gpurun_out/${T}_fc0.json 2> gpurun_out/${T}_fc0.err || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_shapes.py tests/test_gpu_ddp.py tests/test_gpu_timed_step.py -x -v --timeout 120 --timeout-method thread -m gpu -k "frag or linear or ddp or timed" > gpurun_out/${T}_tests.txt 2>&1 || exit $?
echo done
