set -e
mkdir -p gpurun_out
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing --steps 10 --warmup 2"
CLIMSR_DDP_OVERLAP_TEST=1 $B --mode gan > gpurun_out/ov_gtest.json 2> gpurun_out/ov_gtest.err
CLIMSR_DDP_OVERLAP_TEST=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/ov_test.json 2> gpurun_out/ov_test.err
