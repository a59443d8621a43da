# PMC passes over the tokenizer micro-bench (instruction mix, stalls, memory).
cd /root/repo
export TMPDIR=/tmp
N=${1:-2.5e8}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY -d gpurun_out/pmct1 -o tok -- python3 tools/tok_bench.py $N > gpurun_out/pmct1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD -d gpurun_out/pmct2 -o tok -- python3 tools/tok_bench.py $N > gpurun_out/pmct2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d gpurun_out/pmct3 -o tok -- python3 tools/tok_bench.py $N > gpurun_out/pmct3.log 2>&1
