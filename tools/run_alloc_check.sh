# Allocator steadiness: GPU tests touching plans, then C4 both orders and C2 (4-6 steps each).
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-alloc}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_native_gpu.py tests/test_output_gpu.py tests/test_tokenize_gpu.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --steps 4 --rng native > $O/c4n.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --steps 4 > $O/c4r.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 6 > $O/c2.log 2>&1 || exit 4
echo ALLDONE
