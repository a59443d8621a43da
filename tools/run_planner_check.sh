cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py tests/test_balance.py > gpurun_out/t9.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --no-alt-rng > gpurun_out/b9_c2.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --steps 2 --no-alt-rng > gpurun_out/b9_c4.log 2>&1 || exit 3
LDDL_AMD_LIB=lddl_amd/_lib_diag/liblddl_amd.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 1 --warmup 0 --no-alt-rng > gpurun_out/s9.log 2>&1 || exit 4
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_LDS -d gpurun_out/pmc9 -o p -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --no-alt-rng > gpurun_out/pmc9.log 2>&1 || exit 5
