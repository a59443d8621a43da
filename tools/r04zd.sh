set -o pipefail
mkdir -p gpurun_out/r04zd
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py tests/test_native_gpu.py > gpurun_out/r04zd/tests.log 2>&1 || exit 1
echo tests ok
bash tools/run_trace_copies.sh r04zd/trace || exit 1
