set -o pipefail
mkdir -p gpurun_out/r04g
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_native_gpu.py tests/test_output_gpu.py tests/test_balance.py tests/test_segment_gpu.py > gpurun_out/r04g/tests.log 2>&1
echo "tests rc=$?"
B="--steps 3 --no-alt-rng --no-extra-lines --no-segmented-line --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $B > gpurun_out/r04g/new.log 2>&1 || exit 1
LDDL_GATHER_OLD=1 timeout -k 10 300 python -u bench.py $B > gpurun_out/r04g/old.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py $B --rng native > gpurun_out/r04g/new_native.log 2>&1 || exit 1
bash tools/run_trace_copies.sh r04g/trace_new
