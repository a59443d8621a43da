# Native RNG mode: its GPU tests, the replay pair tests, and C2/C4 benches in both modes.
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-native}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_native_gpu.py tests/test_pairs_gpu.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --rng native > $O/c2_native.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --steps 2 --rng native > $O/c4_native.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o b -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --rng native > $O/trace.log 2>&1 || exit 4
echo ALLDONE
