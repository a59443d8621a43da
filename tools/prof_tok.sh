cd /root/repo
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY -d gpurun_out/pmc1 -o tok -- python3 tools/tok_bench.py 2.5e8 > gpurun_out/pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_BRANCH -d gpurun_out/pmc2 -o tok -- python3 tools/tok_bench.py 2.5e8 > gpurun_out/pmc2.log 2>&1
LDDL_AMD_LIB=lddl_amd/_lib_diag/liblddl_amd.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/stamps.log 2>&1
