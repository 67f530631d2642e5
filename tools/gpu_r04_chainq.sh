# Round 4: quick parity of the RDB chain kernel only
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04c}
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_conv.py -k rdb_chain > gpurun_out/${T}_chain.log 2>&1
