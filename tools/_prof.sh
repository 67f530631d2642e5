# Round profile refresh on one MI355X: GPU tests, smoke, PMC traffic passes, kernel-trace stats, bench line.
# usage: bash tools/_prof.sh <tag>      (outputs under gpurun_out/<tag>_*)
set -e
T=${1:-v7}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}f -o run --output-format csv -- $B > gpurun_out/${T}_pmcf.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${T}w -o run --output-format csv -- $B > gpurun_out/${T}_pmcw.log 2>&1
python tools/pmc_traffic.py gpurun_out/${T}f gpurun_out/${T}w gpurun_out/r01_${T}_pmc_traffic "round 1 ${T}: bench.py --steps 2 --warmup 1"
cp gpurun_out/r01_${T}_pmc_traffic.json profiles/
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}s -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing > gpurun_out/${T}_stats.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
