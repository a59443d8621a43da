# Tests + both bench workloads (C2 with the CPU baseline) + tokenizer HBM counters.
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-latest}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench_c2.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --workload c4 --no-cpu-baseline > $O/bench_c4.log 2>&1 || exit 3
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o p -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || exit 4
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o p -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_write.log 2>&1 || exit 5
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o b -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 || exit 6
echo ALLDONE
