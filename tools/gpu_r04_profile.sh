# Round-4 profile refresh on one MI355X: the whole -m gpu suite, smoke, PMC traffic passes (FETCH_SIZE / WRITE_SIZE,
# separate runs), kernel-trace stats of the GAN bench, then the bench line that reads the fresh traffic summary.
# usage: bash tools/gpu_r04_profile.sh <tag: r04_vN>      (outputs under gpurun_out/<tag>_*)
set -o pipefail
T=${1:-r04_v1}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 2 --warmup 1 --median-steps 0 --no-config2 --no-cpu-baseline --no-kernel-timing"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}f -o run --output-format csv -- $B > gpurun_out/${T}_pmcf.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${T}w -o run --output-format csv -- $B > gpurun_out/${T}_pmcw.log 2>&1 || exit $?
python3 tools/pmc_traffic.py gpurun_out/${T}f gpurun_out/${T}w gpurun_out/${T}_gan_pmc_traffic "round 4 ${T}: $B" > /dev/null || exit $?
cp gpurun_out/${T}_gan_pmc_traffic.json gpurun_out/${T}_gan_pmc_traffic.md profiles/
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}s -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --median-steps 0 --no-config2 --no-cpu-baseline --no-kernel-timing > gpurun_out/${T}_stats.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
echo done
