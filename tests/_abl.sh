set -e
mkdir -p gpurun_out
for ab in 0 1 2 4 8 9 6 15; do echo "== ABLATE $ab"; CLIMSR_ABLATE=$ab timeout -k 10 100 python tests/perf_conv.py --rdb-only --reps 50; done > gpurun_out/abl.log 2>&1
