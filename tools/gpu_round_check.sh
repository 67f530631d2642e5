#!/bin/bash
# One gpurun call: GPU parity suite, smoke, pretrain + GAN bench lines, rocprof kernel stats.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_pretrain.json 2> gpurun_out/bench_pretrain.err
timeout -k 10 400 python -u bench.py --mode gan --no-cpu-baseline > gpurun_out/bench_gan.json 2> gpurun_out/bench_gan.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
echo done
