# Round-6 call h: timing attribution of conv_wgrad64_glds_kernel (A/B libraries under ab/: the product kernel with one
# part removed each -- bias MFMAs, in-loop DMA, the per-tile barrier, the MFMAs, the slab epilogue; their results are
# wrong by construction, timing only), alternating with the product build.
set -o pipefail
T=${1:-r06h}
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python -u tools/perf_wgrad64.py product >> gpurun_out/${T}_wg.json 2>&1 || exit $?
  for v in ${VARIANTS:-nodma nomfma noepi nolds noall}; do
    CLIMSR_HIP_LIB=$PWD/ab/lib_wg_$v.so timeout -k 10 200 python -u tools/perf_wgrad64.py $v >> gpurun_out/${T}_wg.json 2>&1 || exit $?
  done
done
echo done
