#!/bin/bash
# One gpurun call (round 3): new / changed GPU parity tests, the whole -m gpu suite, smoke, the bench line (config 3 +
# config 2 sub-record + CPU baselines), config 5 (ESRGAN + RCAN), a kernel-trace summary and the MFMA-busy PMC passes.
# Every GPU step has its own time limit; the steps are chained with && (nothing more runs after a failure).
# usage: bash tests/gpu_r03.sh <tag> [steps...]   steps: new suite smoke bench infer prof mfma traffic (default: all)
T=${1:-v1}
shift
STEPS=${*:-suite smoke}
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
has() { [[ " $STEPS " == *" $1 "* ]]; }
run() {  # name, limit, command...
  local name=$1 lim=$2
  shift 2
  echo "[gpu_r03] $name ($(date +%T))" >&2
  timeout -k 10 "$lim" "$@"
}
set -o pipefail
# pytest: 1 = tests failed (read the log) and the run goes on, unless the log shows a GPU fault; anything else = stop
ok1() { local rc=$?; [ $rc -eq 0 ] || { [ $rc -eq 1 ] && ! grep -q -E "illegal memory access|HIP error|hipError|Memory access fault" "$1"; }; }
{ ! has new || { run new 900 $PYT ${NEW_TESTS:-tests/test_gpu_timed_step.py tests/test_gpu_ddp.py tests/test_gpu_gan.py::test_gan_step_vs_golden tests/test_gpu_configs.py::test_config1_trainer_steps_vs_golden} \
    > gpurun_out/${T}_pytest_new.log 2>&1; ok1 gpurun_out/${T}_pytest_new.log; }; } &&
{ ! has suite || { run suite 1100 $PYT -rP -m gpu tests > gpurun_out/${T}_pytest_gpu.log 2>&1; ok1 gpurun_out/${T}_pytest_gpu.log; }; } &&
{ ! has smoke || run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1; } &&
{ ! has bench || run bench 600 python -u bench.py > gpurun_out/${T}_gan_bench.json 2> gpurun_out/${T}_gan_bench.err; } &&
{ ! has infer || run infer_esrgan 400 python -u bench.py --mode infer --model esrgan --steps 10 --warmup 3 --cpu-seconds 10 \
    > gpurun_out/${T}_infer_esrgan_bench.json 2> gpurun_out/${T}_infer_esrgan.err; } &&
{ ! has infer || run infer_rcan 400 python -u bench.py --mode infer --model rcan --steps 10 --warmup 3 --cpu-seconds 10 \
    > gpurun_out/${T}_infer_rcan_bench.json 2> gpurun_out/${T}_infer_rcan.err; } &&
{ ! has prof || run prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- \
    python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --median-steps 0 --no-config2 > gpurun_out/${T}_prof_bench.json \
    2> gpurun_out/${T}_prof.err; } &&
{ ! has mfma || run mfma 700 python -u tests/pmc_mfma.py gpurun_out/${T}_gan_sq "GAN step (config 3) $T" -- \
    --steps 2 --warmup 1 --median-steps 0 --no-config2 --no-cpu-baseline --no-kernel-timing > gpurun_out/${T}_mfma.log 2>&1; } &&
{ ! has traffic || { run fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}_f -o run --output-format csv -- \
    python3 -u bench.py --steps 2 --warmup 1 --median-steps 0 --no-config2 --no-cpu-baseline --no-kernel-timing > gpurun_out/${T}_f.log 2>&1 &&
  run write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${T}_w -o run --output-format csv -- \
    python3 -u bench.py --steps 2 --warmup 1 --median-steps 0 --no-config2 --no-cpu-baseline --no-kernel-timing > gpurun_out/${T}_w.log 2>&1 &&
  python tests/pmc_traffic.py gpurun_out/${T}_f gpurun_out/${T}_w gpurun_out/${T}_gan_pmc_traffic "GAN step $T" > /dev/null; }; } &&
echo "[gpu_r03] done ($(date +%T))"
