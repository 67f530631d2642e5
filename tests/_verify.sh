set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/verify_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/verify_smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/verify_bench.json 2> gpurun_out/verify_bench.err
timeout -k 10 300 python bench.py --mode gan --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/verify_gan.json 2> gpurun_out/verify_gan.err
