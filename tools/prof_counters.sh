# Instruction-mix / issue / LDS / L2 counters of the C2 bench step (one step, no warmup), one
# rocprofv3 --pmc pass per counter group (gfx950 slots: 8 SQ, 4 TCC per pass).
# usage: bash tools/prof_counters.sh <tag> [extra bench args]
# Summaries: gpurun_out/<tag>/c{1..4}.txt (tools/pmc_summary.py per kernel, mean per dispatch).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-alt-rng --no-segmented-line --steps 1 --warmup 0 $@"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $O/c1 -o p -- $B > $O/c1.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU -d $O/c2 -o p -- $B > $O/c2.log 2>&1 || exit 2
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum -d $O/c3 -o p -- $B > $O/c3.log 2>&1 || exit 3
for k in c1 c2 c3; do python3 tools/pmc_summary.py $(find $O/$k -name "*.db" | head -1) > $O/$k.txt || exit 4; done
echo ALLDONE
