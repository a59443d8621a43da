# PMC passes over one C2 bench step: HBM bytes and wait/issue split of the pairs kernels.
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-pg}
mkdir -p $O
B="python3 bench.py --no-cpu-baseline --steps 1 --warmup 0"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/f -o p -- $B > $O/f.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/w -o p -- $B > $O/w.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY -d $O/s -o p -- $B > $O/s.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d $O/t -o p -- $B > $O/t.log 2>&1 && echo ALLDONE
