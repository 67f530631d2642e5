# Round-2 GPU check (v3): -m gpu tests (incl. config 1 / config 5 parity), smoke, the default bench line,
# FETCH_SIZE / WRITE_SIZE PMC passes of the GAN step (separate runs), rocprofv3 kernel stats of the GAN step.
# Stops at the first step that crashes / times out (anything but pass or plain test failures).
T=${1:-v3}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 540 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
echo "smoke ok"
timeout -k 10 300 python3 -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
echo "bench ok"
B="python3 bench.py --steps 2 --warmup 1 --median-steps 0 --no-config2 --no-cpu-baseline --no-kernel-timing"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}f -o run --output-format csv -- $B > gpurun_out/${T}_pmcf.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${T}w -o run --output-format csv -- $B > gpurun_out/${T}_pmcw.log 2>&1 || exit $?
python tests/pmc_traffic.py gpurun_out/${T}f gpurun_out/${T}w gpurun_out/r02_${T}_gan_pmc_traffic "round 2 ${T}: GAN step, bench.py --steps 2 --warmup 1" > gpurun_out/${T}_pmc.md || exit $?
echo "pmc ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}s -o run -- python3 -u bench.py --no-cpu-baseline --no-config2 --no-kernel-timing --steps 20 --warmup 5 --median-steps 0 > gpurun_out/${T}_prof.json 2> gpurun_out/${T}_prof.err || exit $?
echo "prof ok"
