# SQ / TCC counter passes over tools/perf_vgg.py under each CLIMSR_CONV_DMA setting (args: tag)
T=${1:-sv}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for D in 0 1; do
  export CLIMSR_CONV_DMA=$D
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_kt$D -o run --output-format csv -- python3 tools/perf_vgg.py > gpurun_out/${T}_kt$D.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS -d gpurun_out/${T}1_$D -o run --output-format csv -- python3 tools/perf_vgg.py > gpurun_out/${T}1_$D.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/${T}2_$D -o run --output-format csv -- python3 tools/perf_vgg.py > gpurun_out/${T}2_$D.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d gpurun_out/${T}3_$D -o run --output-format csv -- python3 tools/perf_vgg.py > gpurun_out/${T}3_$D.log 2>&1 || exit $?
  python3 tools/sq_summary.py gpurun_out/${T}1_$D gpurun_out/${T}2_$D gpurun_out/${T}3_$D > gpurun_out/${T}_summary_$D.txt
done
