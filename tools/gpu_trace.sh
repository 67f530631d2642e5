# A kernel trace of a short GAN bench (rocprofv3 --kernel-trace, csv) summarised by tools/trace_summary.py: per-step
# kernel time, gaps between kernels, and where the device copies sit.   usage: bash tools/gpu_trace.sh <tag>
set -o pipefail
T=${1:-trace}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${T}_t -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --median-steps 0 --no-config2 --no-cpu-baseline --no-kernel-timing > gpurun_out/${T}_trace.log 2>&1 || exit $?
python3 tools/trace_summary.py gpurun_out/${T}_t > gpurun_out/${T}_trace_summary.txt || exit $?
rm -rf gpurun_out/${T}_t
echo done
