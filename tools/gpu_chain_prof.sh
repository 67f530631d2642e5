# RDB chain micro-benchmark (B=32, 64x64, tools/perf_conv.py --rdb-only): timing, then two SQ counter passes
set -o pipefail
mkdir -p gpurun_out
T=${1:-chq}
timeout -k 10 120 python3 tools/perf_conv.py --rdb-only --reps 20 > gpurun_out/${T}_time.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="python3 tools/perf_conv.py --rdb-only --reps 5"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS -d gpurun_out/${T}1 -o run --output-format csv -- $P > gpurun_out/${T}1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/${T}2 -o run --output-format csv -- $P > gpurun_out/${T}2.log 2>&1 || exit $?
python3 tools/sq_summary.py gpurun_out/${T}1 gpurun_out/${T}2 > gpurun_out/${T}_sq.txt
