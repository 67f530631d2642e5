set -e
mkdir -p gpurun_out
for ab in 0 1 2 4 8 6 3; do echo "== ABLATE $ab"; CLIMSR_ABLATE=$ab timeout -k 10 100 python tests/perf_conv.py --rdb-only; done > gpurun_out/abl.log 2>&1
for pc in 1 3 4; do echo "== PER_CU $pc"; CLIMSR_N16_PER_CU=$pc timeout -k 10 100 python tests/perf_conv.py --rdb-only; done >> gpurun_out/abl.log 2>&1
