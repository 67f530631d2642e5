# Round profile of the build the driver benches, on one MI355X: the whole -m gpu suite, smoke, then for the GAN step
# and both config-5 inference models: FETCH_SIZE / WRITE_SIZE PMC passes (separate runs) -> profiles/<tag>_<mode>_pmc_
# traffic.{json,md} (with the library sha256 bench.py matches), kernel-trace stats -> profiles/<tag>_<mode>_kernel_stats.csv
# (+ .meta.json), and the bench lines.
# usage: CLIMSR_GIT_HEAD=$(git rev-parse HEAD) bash tools/gpu_profile.sh <tag: rNN_vM> [part: gan | infer]
#   (gan: the suite, smoke, the GAN step's profiles and bench line; infer: config 5's; one gpurun call each)
set -o pipefail
T=${1:-r05_v1}
PART=${2:-gan}
mkdir -p gpurun_out
export CLIMSR_GIT_HEAD
if [ $PART = gan ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || exit $?
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
  MODES=gan
else
  MODES="esrgan rcan"
fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for mode in $MODES; do
  case $mode in
    gan) B="python3 bench.py --steps 2 --warmup 1 --median-steps 0 --no-config2 --no-cpu-baseline --no-kernel-timing"
         S="python3 bench.py --steps 10 --warmup 2 --median-steps 0 --no-config2 --no-cpu-baseline --no-kernel-timing" ;;
    *) B="python3 bench.py --mode infer --model $mode --steps 2 --warmup 1 --median-steps 0 --no-cpu-baseline --no-kernel-timing"
       S="python3 bench.py --mode infer --model $mode --steps 5 --warmup 1 --median-steps 0 --no-cpu-baseline --no-kernel-timing" ;;
  esac
  M=$mode; [ $mode != gan ] && M=infer_$mode
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}_${M}_f -o run --output-format csv -- $B > gpurun_out/${T}_${M}_pmcf.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${T}_${M}_w -o run --output-format csv -- $B > gpurun_out/${T}_${M}_pmcw.log 2>&1 || exit $?
  python3 tools/pmc_traffic.py gpurun_out/${T}_${M}_f gpurun_out/${T}_${M}_w gpurun_out/${T}_${M}_pmc_traffic "${T}: $B" > /dev/null || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_${M}_s -o run --output-format csv -- $S > gpurun_out/${T}_${M}_stats.log 2>&1 || exit $?
  python3 tools/prof_record.py gpurun_out/${T}_${M}_s gpurun_out/${T}_${M}_kernel_stats.csv "$S" || exit $?
  rm -rf gpurun_out/${T}_${M}_f gpurun_out/${T}_${M}_w gpurun_out/${T}_${M}_s
done
if [ $PART = gan ]; then
  bash tools/gpu_sq.sh ${T}_gan_sq > gpurun_out/${T}_gan_sq.log 2>&1 || exit $?
  rm -rf gpurun_out/${T}_gan_sq1 gpurun_out/${T}_gan_sq2
  timeout -k 10 400 python3 -u bench.py > gpurun_out/${T}_gan_bench.json 2> gpurun_out/${T}_gan_bench.err || exit $?
else
  timeout -k 10 300 python3 -u bench.py --mode infer --model rcan > gpurun_out/${T}_infer_rcan_bench.json 2> gpurun_out/${T}_infer_rcan_bench.err || exit $?
  timeout -k 10 300 python3 -u bench.py --mode infer --model esrgan > gpurun_out/${T}_infer_esrgan_bench.json 2> gpurun_out/${T}_infer_esrgan_bench.err || exit $?
fi
echo done
