# SQ counter passes over the RDB micro-benchmark (tools/perf_conv.py --rdb-only), summarised by tools/sq_summary.py.
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="python3 tools/perf_conv.py --rdb-only --reps 5"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS -d gpurun_out/sqc1 -o run --output-format csv -- $P > gpurun_out/sqc1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/sqc2 -o run --output-format csv -- $P > gpurun_out/sqc2.log 2>&1 || exit $?
python3 tools/sq_summary.py gpurun_out/sqc1 gpurun_out/sqc2 > gpurun_out/sq_chain.txt
