# Round 4: the CLIMSR_CONV_DMA_PW=1 route (HRconv / upconv1/2 / VGG conv1_2 on the LDS-DMA conv) through the WHOLE
# -m gpu suite (no -x: every test runs), then the GAN-step A/B against the default conv_pw route.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04a}
CLIMSR_CONV_DMA_PW=1 timeout -k 10 420 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pw_pytest.log 2>&1
rc=$?; echo "pytest rc $rc" >> gpurun_out/${T}_pw_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2; do
  CLIMSR_CONV_DMA_PW=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_pw_$r.json 2>> gpurun_out/${T}_bench.err || exit $?
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_nopw_$r.json 2>> gpurun_out/${T}_bench.err || exit $?
done
