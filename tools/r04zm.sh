set -o pipefail
mkdir -p gpurun_out/r04zm
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04zm/tests.log 2>&1 || exit 1
echo tests ok
bash tools/run_trace_copies.sh r04zm/trace || exit 1
