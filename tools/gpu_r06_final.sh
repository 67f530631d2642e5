# Round-6 final records: config-5 profiles of the committed build (gpu_profile.sh infer part), then the default bench
# line (GAN step, config 3) now that the build's PMC traffic summary is under profiles/.
set -o pipefail
T=${1:-r06_v3}
bash tools/gpu_profile.sh $T infer || exit $?
timeout -k 10 400 python3 -u bench.py > gpurun_out/${T}_gan_bench_default.json 2> gpurun_out/${T}_gan_bench_default.err || exit $?
echo done
