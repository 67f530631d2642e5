# SQ counter passes over a short GAN bench (two --pmc runs of <= 8 SQ counters each), summarised per kernel.
T=${1:-sq}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 2 --warmup 1 --median-steps 0 --no-config2 --no-cpu-baseline --no-kernel-timing"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS -d gpurun_out/${T}1 -o run --output-format csv -- $B > gpurun_out/${T}1.log 2>&1 || exit $?
echo pass1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/${T}2 -o run --output-format csv -- $B > gpurun_out/${T}2.log 2>&1 || exit $?
echo pass2
python3 tools/sq_summary.py gpurun_out/${T}1 gpurun_out/${T}2 > gpurun_out/${T}_summary.txt
