# A/B timing of env switches in one GPU call: perf_diag + the bench step under each setting (args: tag setting...),
# a setting is NAME=VALUE or "base"
set -o pipefail
mkdir -p gpurun_out
T=$1; shift
for v in "$@"; do
  for r in 1 2; do
    if [ $v = base ]; then e=CLIMSR_AB_NONE=1; else e=$v; fi
    env $e timeout -k 10 120 python -u tests/perf_diag.py "$v" >> gpurun_out/${T}_diag.jsonl 2>> gpurun_out/${T}_diag.err || exit $?
    env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --steps 20 --warmup 5 > gpurun_out/${T}_bench_${v//=/_}_$r.json 2>> gpurun_out/${T}_bench.err || exit $?
  done
done
