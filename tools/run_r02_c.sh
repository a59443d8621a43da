cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_collate_gpu.py tests/test_loader.py tests/test_balance.py tests/test_output_gpu.py > $O/gpu_tests.log 2>&1
timeout -k 10 600 python -u bench.py --workload c5 --steps 200 --warmup 20 > $O/bench_c5.log 2>&1 || exit 3
timeout -k 10 600 python -u bench.py --workload c4 --no-cpu-baseline --no-segmented-line --no-alt-rng > $O/bench_c4.log 2>&1 || exit 4
echo ALLDONE
