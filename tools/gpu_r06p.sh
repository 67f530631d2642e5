# Round-6 call p: run-to-run spread of the final build on one box (three GAN bench lines and two config-5 RCAN lines
# back to back), to set against the box-to-box spread of the round's calls.
set -o pipefail
T=${1:-r06p}
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-config2 > gpurun_out/${T}_gan_$i.json 2> gpurun_out/${T}_gan_$i.err || exit $?
done
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --mode infer --no-cpu-baseline > gpurun_out/${T}_infer_$i.json 2> gpurun_out/${T}_infer_$i.err || exit $?
done
echo done
