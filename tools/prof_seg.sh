# SQ PMC passes over tools/seg_bench.py (segmentation only)
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
B="python3 tools/seg_bench.py 0.5"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY -d $O/m1 -o p -- $B > $O/m1.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS -d $O/m2 -o p -- $B > $O/m2.log 2>&1 &&
python3 tools/pmc_summary.py $(find $O/m1 -name "*.db") > $O/mix1.txt &&
python3 tools/pmc_summary.py $(find $O/m2 -name "*.db") > $O/mix2.txt && echo ALLDONE
