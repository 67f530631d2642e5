# Round 5, call p: fc.0 weight copy in fragment order (forward / data gradient / AdamW mirror) and the two D backwards'
# fc.0 weight gradients in one launch: the new parity tests, the fc.0 microbenchmark, the whole -m gpu suite, then the
# GAN step alternating both on / merged weight gradient only / neither on this box.   usage: bash tools/gpu_r05p.sh <tag>
set -o pipefail
mkdir -p gpurun_out
T=${1:-r05p}
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_shapes.py -x -v --timeout 120 --timeout-method thread -m gpu -k "frag or linear" > gpurun_out/${T}_frag_tests.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/bench_linear_fc0.py > gpurun_out/${T}_fc0.json 2> gpurun_out/${T}_fc0.err || exit $?
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/${T}_pytest_gpu.txt 2>&1 || exit $?
B="python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5"
for i in 1 2; do
  CLIMSR_FC0_FRAG=1 CLIMSR_FC0_WGRAD_MERGE=1 timeout -k 10 300 $B > gpurun_out/${T}_bench_both_$i.json 2> gpurun_out/${T}_bench_both_$i.err || exit $?
  CLIMSR_FC0_FRAG=0 CLIMSR_FC0_WGRAD_MERGE=1 timeout -k 10 300 $B > gpurun_out/${T}_bench_merge_$i.json 2> gpurun_out/${T}_bench_merge_$i.err || exit $?
  CLIMSR_FC0_FRAG=0 CLIMSR_FC0_WGRAD_MERGE=0 timeout -k 10 300 $B > gpurun_out/${T}_bench_none_$i.json 2> gpurun_out/${T}_bench_none_$i.err || exit $?
done
echo done
