set -o pipefail
mkdir -p gpurun_out/r04b
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_native_gpu.py tests/test_pairs_gpu.py tests/test_balance.py tests/test_output_gpu.py > gpurun_out/r04b/tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04b/prof_native -o native -- python3 bench.py --rng native --steps 2 --warmup 1 --no-alt-rng --no-extra-lines --no-segmented-line --no-cpu-baseline > gpurun_out/r04b/native.log 2>&1 || exit 1
echo native done
