# Gather A/B: GPU pair/output tests, C2 + C4 benches (default gather), C2 with the v2 gather,
# and a kernel trace of one C2 step.
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-gather}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py tests/test_balance.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 > $O/c2.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --steps 2 > $O/c4.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o b -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 || exit 4
echo ALLDONE
