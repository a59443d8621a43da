# Per-kernel counters of one C2 bench step (no warmup): SQ instruction mix / issue / LDS / L2 and
# HBM bytes, one rocprofv3 --pmc pass per counter group (gfx950 slots: 8 SQ, 4 TCC per pass;
# FETCH_SIZE and WRITE_SIZE in passes of their own), plus a kernel trace of the same command.
# usage: bash tools/prof_counters.sh <tag> [extra bench args]
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O/pmc
B="python3 bench.py --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines --steps 1 --warmup 0 $@"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $O/pmc/c1 -o p -- $B > $O/c1.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU -d $O/pmc/c2 -o p -- $B > $O/c2.log 2>&1 || exit 2
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum -d $O/pmc/c3 -o p -- $B > $O/c3.log 2>&1 || exit 3
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc/fetch -o p -- $B > $O/fetch.log 2>&1 || exit 4
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc/write -o p -- $B > $O/write.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o k -- $B > $O/trace.log 2>&1 || exit 6
for k in c1 c2 c3 fetch write; do python3 tools/pmc_summary.py $(find $O/pmc/$k -name "*.db" | head -1) > $O/$k.txt || exit 7; done
echo ALLDONE
