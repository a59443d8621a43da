cd /root/repo
export TMPDIR=/tmp
LDDL_AMD_LIB=lddl_amd/_lib_diag/liblddl_amd.so timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/s10.log 2>&1 || exit 4
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/trace10 -o b -- python3 bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/trace10.log 2>&1 || exit 5
