# PMC passes over one bench step (4 GiB): instruction mix of the planner and tokenizer kernels.
cd /root/repo
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --batch-bytes 4294967296"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY -d gpurun_out/pmcp1 -o p -- $B > gpurun_out/pmcp1.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS -d gpurun_out/pmcp2 -o p -- $B > gpurun_out/pmcp2.log 2>&1
